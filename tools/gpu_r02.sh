#!/bin/bash
# Round-2 GPU routine: focused test files (verbose, prints), then the whole -m gpu suite, then a
# short bench.  usage: bash tools/gpu_r02.sh "tests/a.py tests/b.py" [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
FOCUS=${1:-}; shift
if [ -n "$FOCUS" ]; then
  timeout -k 10 600 python -u -m pytest $FOCUS -x -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/focus.log 2>&1
  rc=$?
  grep -E "rel|PASS|FAIL|Error|error|assert|step|scale|swap|validation|reuse" gpurun_out/focus.log | tail -60
  [ $rc = 0 ] || exit 1
fi
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?
tail -3 gpurun_out/tests.log
[ $rc = 0 ] || exit 1
timeout -k 10 300 python bench.py --skip-cpu --steps 30 "$@" > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-400
