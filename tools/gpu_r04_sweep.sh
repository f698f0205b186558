#!/bin/bash
# round 4: training-step A/B over tuning knobs after the round's kernel changes
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
for e in "ENCDIFF_GN_MIN_SLICE=8192" "ENCDIFF_GN_MIN_SLICE=4096" "ENCDIFF_GN_MIN_SLICE=16384" "ENCDIFF_SPLIT_FOLD=0" "ENCDIFF_GN_MIN_SLICE=8192" "ENCDIFF_GN_MIN_SLICE=4096"; do
  env $e timeout -k 10 400 python bench.py --skip-cpu --skip-ddim --steps 30 > gpurun_out/sw.log 2>&1 || { tail -5 gpurun_out/sw.log; exit 1; }
  echo "$e: $(tail -1 gpurun_out/sw.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), round(d['value']))")"
done
