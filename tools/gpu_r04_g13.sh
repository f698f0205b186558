#!/bin/bash
# round 4: GroupNorm backward code-size A/B (rows per load batch 4 / 2 / 1)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "groupnorm" --timeout 200 --timeout-method thread > gpurun_out/gn13.log 2>&1 || { tail -30 gpurun_out/gn13.log; exit 1; }
tail -1 gpurun_out/gn13.log
for v in default gnu2 gnu1; do
  if [ $v = default ]; then L=""; else L=encdiff_amd/_ab/libencdiff_hip_$v.so; fi
  env ${L:+ENCDIFF_LIB=$L} timeout -k 10 200 python -u tools/gn_bench.py > gpurun_out/gn_bench_$v.txt 2>&1 || { tail -5 gpurun_out/gn_bench_$v.txt; exit 1; }
  echo "== $v"; grep H= gpurun_out/gn_bench_$v.txt
done
