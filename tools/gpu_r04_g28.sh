#!/bin/bash
# round 4: wave-per-slice GroupNorm forward for sampling batches -- tests, DDIM A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "groupnorm or st_head or st_tail" --timeout 200 --timeout-method thread > gpurun_out/gn28.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/gn28.log | head; tail -30 gpurun_out/gn28.log; exit 1; }
tail -1 gpurun_out/gn28.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_ldm.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/unet28.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/unet28.log | head; tail -20 gpurun_out/unet28.log; exit 1; }
tail -1 gpurun_out/unet28.log
bash tools/ddim_env_ab.sh 8 100 "ENCDIFF_GN_WAVE_MAX_B=0" "ENCDIFF_GN_WAVE_MAX_B=32" "ENCDIFF_GN_WAVE_MAX_B=0" "ENCDIFF_GN_WAVE_MAX_B=32"
