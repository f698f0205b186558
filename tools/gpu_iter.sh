#!/bin/bash
# GPU-box iteration: focused tests (pytest -k / node ids, verbose), then a short graph bench (optional
# env A/B arms).   usage: TESTS="tests/x.py::t tests/y.py" bash tools/gpu_iter.sh ["ENV=1" "ENV=0" ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -v -s --timeout 200 --timeout-method thread > gpurun_out/iter_tests.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR|rel|Error|assert" gpurun_out/iter_tests.log | tail -60
  [ $rc = 0 ] || { tail -30 gpurun_out/iter_tests.log; exit 1; }
fi
[ "$NOBENCH" = 1 ] && exit 0
ARMS=("$@"); [ ${#ARMS[@]} = 0 ] && ARMS=("X=0")
for e in "${ARMS[@]}"; do
  for rep in 1 2; do
    env $e timeout -k 10 200 python bench.py --skip-cpu --skip-ref-api --skip-ddim --steps 50 > gpurun_out/iter_bench.log 2>&1 || { tail -15 gpurun_out/iter_bench.log; exit 1; }
    echo "$e: $(tail -1 gpurun_out/iter_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms/step", round(d["value"]), "imgs/s", "frac", round(d["roofline"]["frac"],4))')"
  done
done
