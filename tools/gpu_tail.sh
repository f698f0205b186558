#!/bin/bash
# Fused SpatialTransformer tail: focused parity tests, DDIM B=8 rate with the tail fused / unfused.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_ldm.py -x -v -s -m gpu --timeout 200 --timeout-method thread > gpurun_out/tail_tests.log 2>&1
rc=$?
grep -E "fused|rel|passed|failed|Error|error|assert" gpurun_out/tail_tests.log | tail -30
[ $rc = 0 ] || exit 1
for v in 1 0; do
  ENCDIFF_ST_TAIL=$v timeout -k 10 120 python tools/ddim_prof.py --batch 8 --steps 200 2>&1 | grep steps/s | sed "s/^/tail=$v /" || exit 1
done
