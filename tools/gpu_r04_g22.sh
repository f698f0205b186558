#!/bin/bash
# round 4: attention backward dS^T chunk (keys per chunk -> workgroups per CU) A/B at dh 8
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
for k in 64 32 16 64 32 16; do
  ENCDIFF_ATTN_KCHUNK=$k timeout -k 10 200 python -u tools/attn_bench.py --only 8 > gpurun_out/attn_k$k.txt 2>&1 || { tail -5 gpurun_out/attn_k$k.txt; exit 1; }
  echo "KCHUNK=$k: $(grep 'sk=256' gpurun_out/attn_k$k.txt)"
done
