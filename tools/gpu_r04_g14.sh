#!/bin/bash
# round 4: attention forward score-bound path + backward dP-from--D accumulators, GroupNorm
# backward slab specialisation: full op tests, attention and GroupNorm timing
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu --timeout 200 --timeout-method thread -s > gpurun_out/ops14.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/ops14.log | head -20; tail -30 gpurun_out/ops14.log; exit 1; }
tail -1 gpurun_out/ops14.log; grep "score bound" gpurun_out/ops14.log
timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/attn_bench.txt 2>&1 || { tail -5 gpurun_out/attn_bench.txt; exit 1; }
cat gpurun_out/attn_bench.txt | grep -v amdgpu.ids
timeout -k 10 200 python -u tools/gn_bench.py > gpurun_out/gn_bench.txt 2>&1 || { tail -5 gpurun_out/gn_bench.txt; exit 1; }
grep H= gpurun_out/gn_bench.txt
