#!/bin/bash
# Round-4 GPU routine: focused test files (verbose, prints), optional smoke, the whole -m gpu
# suite, a short bench.  usage: bash tools/gpu_r04.sh "tests/a.py tests/b.py" [smoke|nosmoke] [full|nofull] [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
FOCUS=${1:-}; SMOKE=${2:-nosmoke}; FULL=${3:-full}; shift 3
if [ -n "$FOCUS" ]; then
  timeout -k 10 900 python -u -m pytest $FOCUS -x -v -s -m gpu --timeout 600 --timeout-method thread > gpurun_out/focus.log 2>&1
  rc=$?
  grep -E "rel|PASS|FAIL|Error|error|assert|step|scale|swap|B=|smoke|passed|failed" gpurun_out/focus.log | tail -60
  [ $rc = 0 ] || exit 1
fi
if [ "$SMOKE" = smoke ]; then
  timeout -k 10 600 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
  tail -3 gpurun_out/smoke.log
fi
if [ "$FULL" = full ]; then
  timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/tests.log 2>&1
  rc=$?
  tail -3 gpurun_out/tests.log
  [ $rc = 0 ] || exit 1
fi
if [ "$1" != "nobench" ]; then
  timeout -k 10 400 python bench.py --skip-cpu --steps 30 "$@" > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
  tail -1 gpurun_out/bench.log | cut -c1-600
fi
