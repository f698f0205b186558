#!/bin/bash
# round 4: GroupNorm backward -- norm.hip at -ffp-contract=on (default) vs fast, per-shape timing
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "groupnorm" --timeout 200 --timeout-method thread > gpurun_out/gn21.log 2>&1 || { tail -30 gpurun_out/gn21.log; exit 1; }
tail -1 gpurun_out/gn21.log
for v in default nfast default nfast; do
  if [ $v = default ]; then L=""; else L=encdiff_amd/_ab/libencdiff_hip_$v.so; fi
  env ${L:+ENCDIFF_LIB=$L} timeout -k 10 200 python -u tools/gn_bench.py > gpurun_out/gn_bench_$v.txt 2>&1 || { tail -5 gpurun_out/gn_bench_$v.txt; exit 1; }
  echo "== $v"; grep H= gpurun_out/gn_bench_$v.txt | cut -c1-75
done
