#!/bin/bash
# Bench A/B over environment settings (graph step, no CPU / DDIM legs), two runs each:
#   bash tools/bench_ab.sh "A=0" "A=1 B=2"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for e in "$@"; do
  for rep in 1 2; do
    env $e timeout -k 10 200 python bench.py --skip-cpu --skip-ddim --steps 50 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
    echo "$e: $(tail -1 gpurun_out/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms/step", round(d["value"]), "imgs/s")')"
  done
done
