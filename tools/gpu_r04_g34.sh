#!/bin/bash
# round 4: attention dh 8 forward A/B (key-loop unroll, tiles per task)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
for v in default u4 u1 nt2 nt8 default u4; do
  if [ $v = default ]; then L=""; else L=encdiff_amd/_ab/libencdiff_hip_$v.so; fi
  env ${L:+ENCDIFF_LIB=$L} timeout -k 10 200 python -u tools/attn_bench.py --only 8 > gpurun_out/attn_$v.txt 2>&1 || { tail -5 gpurun_out/attn_$v.txt; exit 1; }
  echo "$v: $(grep 'sk=256' gpurun_out/attn_$v.txt) | $(grep 'sk= 20' gpurun_out/attn_$v.txt | cut -c20-)"
done
