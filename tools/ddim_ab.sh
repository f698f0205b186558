#!/bin/bash
# DDIM B=8 (S=200) steps/s A/B over environment settings, two runs each (bench.py's DDIM leg).
#   bash tools/ddim_ab.sh "A=0" "A=1"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for e in "$@"; do
  for rep in 1 2; do
    env $e timeout -k 10 300 python bench.py --skip-cpu --skip-ref-api --steps 3 --warmup 2 > gpurun_out/ddim_ab.log 2>&1 || { tail -5 gpurun_out/ddim_ab.log; exit 1; }
    echo "$e: $(tail -1 gpurun_out/ddim_ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ddim_steps_per_sec"]["value"],1), "DDIM B=8 steps/s;", round(d["ddim_steps_per_sec_b128"]["value"],1), "B=128 eta=1;", round(d["ms_per_step"],3), "ms/train step")')"
  done
done
