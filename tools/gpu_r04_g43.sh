#!/bin/bash
# round 4: LayerNorm in the consuming linear's A staging (inference, c > 128) -- op + model tests, DDIM A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "layernorm_in_staging or linear or layernorm" --timeout 200 --timeout-method thread > gpurun_out/o43.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/o43.log | head; tail -30 gpurun_out/o43.log; exit 1; }
tail -1 gpurun_out/o43.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_ldm.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/u43.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/u43.log | head; tail -20 gpurun_out/u43.log; exit 1; }
tail -1 gpurun_out/u43.log
bash tools/ddim_env_ab.sh 8 200 "ENCDIFF_LNA=0" "ENCDIFF_LNA=1" "ENCDIFF_LNA=0" "ENCDIFF_LNA=1"
