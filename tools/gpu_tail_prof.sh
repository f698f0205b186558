#!/bin/bash
# DDIM B=8 with the fused SpatialTransformer tail: rate per widest fused level, kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
for mc in 0 64 128 256; do
  ENCDIFF_ST_TAIL_MAXC=$mc timeout -k 10 120 python tools/ddim_prof.py --batch 8 --steps 200 2>&1 | grep steps/s | sed "s/^/maxc=$mc /" || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/tailprof -o run -- python3 $R/tools/ddim_prof.py --batch 8 --steps 50 > $R/gpurun_out/tailprof.log 2>&1 || exit 1
cd $R && python tools/rocpd_stats.py $(find gpurun_out/tailprof -name "*.db" | head -1) --last 19000 --per 50 --top 25 | cut -c1-170
rm -rf gpurun_out/tailprof
