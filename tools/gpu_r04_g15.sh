#!/bin/bash
# round 4: attention SQ counters (dh 8), UNet + LDM GPU tests, short bench
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
bash tools/attn_pmc.sh 8 > gpurun_out/attn_pmc8.txt 2>&1 || { tail -5 gpurun_out/attn_pmc8.txt; exit 1; }
cat gpurun_out/attn_pmc8.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_ldm.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/unet15.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/unet15.log | head; tail -20 gpurun_out/unet15.log; exit 1; }
tail -1 gpurun_out/unet15.log
timeout -k 10 400 python bench.py --skip-cpu --steps 30 > gpurun_out/b15.log 2>&1 || { tail -5 gpurun_out/b15.log; exit 1; }
tail -1 gpurun_out/b15.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['ddim_steps_per_sec'], d['ddim_steps_per_sec_b128'], d.get('ddim_log_images_s'))"
