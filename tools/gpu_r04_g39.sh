#!/bin/bash
# round 4: fused transformer tail at c = 256 (ENCDIFF_ST_TAIL_MAXC=256) -- parity + bench / DDIM A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
ENCDIFF_ST_TAIL_MAXC=256 timeout -k 10 600 python -u -m pytest tests/test_gpu_unet.py -x -q -m gpu -k "oracle or fixture" --timeout 300 --timeout-method thread > gpurun_out/t39.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/t39.log | head; tail -20 gpurun_out/t39.log; exit 1; }
tail -1 gpurun_out/t39.log
for v in 128 256 128 256; do
  ENCDIFF_ST_TAIL_MAXC=$v timeout -k 10 400 python bench.py --skip-cpu --skip-ddim --steps 30 > gpurun_out/b39_$v.log 2>&1 || { tail -5 gpurun_out/b39_$v.log; exit 1; }
  echo "MAXC=$v: $(tail -1 gpurun_out/b39_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), round(d['value']))")"
done
bash tools/ddim_env_ab.sh 8 200 "ENCDIFF_ST_TAIL_MAXC=128" "ENCDIFF_ST_TAIL_MAXC=256" "ENCDIFF_ST_TAIL_MAXC=128" "ENCDIFF_ST_TAIL_MAXC=256"
