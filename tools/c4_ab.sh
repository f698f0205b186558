#!/bin/bash
# configs[4] (CelebA 128x128) training-step A/B over environment settings, two runs each.
#   bash tools/c4_ab.sh "ENCDIFF_ATTN_FP8=0" "ENCDIFF_ATTN_FP8=1"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for e in "$@"; do
  for rep in 1 2; do
    env $e timeout -k 10 300 python bench.py --config celeba128 --skip-cpu --skip-ref-api --skip-ddim --steps 10 --warmup 3 > gpurun_out/c4_ab.log 2>&1 || { tail -5 gpurun_out/c4_ab.log; exit 1; }
    echo "$e: $(tail -1 gpurun_out/c4_ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms/step", round(d["value"]), "imgs/s")')"
  done
done
