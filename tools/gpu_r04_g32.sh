#!/bin/bash
# round 4: UNet optimizer on a side stream under the cond-stage backward -- trainer tests, bench A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_ldm.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tr32.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/tr32.log | head; tail -20 gpurun_out/tr32.log; exit 1; }
tail -1 gpurun_out/tr32.log
for v in 1 0 1 0; do
  ENCDIFF_OPT_OVERLAP=$v timeout -k 10 400 python bench.py --skip-cpu --skip-ddim --steps 40 > gpurun_out/b32_$v.log 2>&1 || { tail -5 gpurun_out/b32_$v.log; exit 1; }
  echo "OPT_OVERLAP=$v: $(tail -1 gpurun_out/b32_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), round(d['value']), d['loss_simple_last'])")"
done
