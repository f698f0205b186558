#!/bin/bash
# GPU-box routine for iteration: optional focused test file (verbose), the full -m gpu suite,
# then a short graph bench.  usage: bash tools/gpu_quick.sh [focus_test_file] [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
FOCUS=${1:-}; shift
if [ -n "$FOCUS" ]; then
  timeout -k 10 300 python -u -m pytest "$FOCUS" -x -q -s --timeout 120 --timeout-method thread > gpurun_out/focus.log 2>&1
  rc=$?
  grep -E "rel|passed|failed|Error|error|assert" gpurun_out/focus.log | tail -40
  [ $rc = 0 ] || exit 1
fi
timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?
tail -3 gpurun_out/tests.log
[ $rc = 0 ] || exit 1
timeout -k 10 200 python bench.py --skip-cpu --skip-ddim --steps 30 "$@" > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-240
