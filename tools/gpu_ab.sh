#!/bin/bash
# Full -m gpu suite, then the default bench (graph, no CPU/DDIM legs) with an env A/B:
#   bash tools/gpu_ab.sh "ENV=0" "ENV=1"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?
grep -E "rel|passed|failed|Error|assert" gpurun_out/tests.log | tail -12
[ $rc = 0 ] || exit 1
for e in "$@"; do
  for rep in 1 2; do
    env $e timeout -k 10 200 python bench.py --skip-cpu --skip-ddim --steps 50 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    echo "$e: $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms/step", round(d["value"]), "imgs/s")')"
  done
done
