#!/bin/bash
# round 4: DDIM whole-loop graph with the FiLM table / K,V computed once per loop -- tests, A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ldm.py tests/test_gpu_unet.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ldm35.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/ldm35.log | head; tail -30 gpurun_out/ldm35.log; exit 1; }
tail -1 gpurun_out/ldm35.log
bash tools/ddim_env_ab.sh 8 200 "ENCDIFF_DDIM_HOIST=0" "ENCDIFF_DDIM_HOIST=1" "ENCDIFF_DDIM_HOIST=0" "ENCDIFF_DDIM_HOIST=1"
