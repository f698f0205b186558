#!/bin/bash
# round 4: GN_FIN bitwise diagnosis across norm.hip variants
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
for v in default slabu4 normprev; do
  if [ $v = default ]; then L=""; else L=encdiff_amd/_ab/libencdiff_hip_$v.so; fi
  env ${L:+ENCDIFF_LIB=$L} timeout -k 10 200 python tools/gnfin_diag.py > gpurun_out/gnfin_$v.txt 2>&1 || { tail -5 gpurun_out/gnfin_$v.txt; exit 1; }
  echo "== $v"; sed -n 2,6p gpurun_out/gnfin_$v.txt
done
