#!/bin/bash
# round 4: GroupNorm backward prefetch -- tests + per-shape A/B (tools/gn_bench.py)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "groupnorm" --timeout 200 --timeout-method thread > gpurun_out/gn12.log 2>&1 || { tail -30 gpurun_out/gn12.log; exit 1; }
tail -1 gpurun_out/gn12.log
timeout -k 10 200 python -u tools/gn_bench.py > gpurun_out/gn_bench_pre1.txt 2>&1 || { tail -5 gpurun_out/gn_bench_pre1.txt; exit 1; }
ENCDIFF_LIB=encdiff_amd/_ab/libencdiff_hip_gnpre0.so timeout -k 10 200 python -u tools/gn_bench.py > gpurun_out/gn_bench_pre0.txt 2>&1 || { tail -5 gpurun_out/gn_bench_pre0.txt; exit 1; }
echo "== prefetch"; cat gpurun_out/gn_bench_pre1.txt; echo "== no prefetch"; cat gpurun_out/gn_bench_pre0.txt
