#!/bin/bash
# Eager kernel-trace window of the bench step (10 steps) -> gpurun_out/<tag>_window.txt
# usage: bash tools/prof_window.sh TAG   (environment passes through to bench.py)
set -o pipefail
TAG=${1:-w}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --skip-ddim --skip-cpu --skip-ref-api --no-graph > $R/gpurun_out/${TAG}_prof.log 2>&1 || { echo "prof failed"; exit 1; }
cd $R
T=$(find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" | head -1)
python tools/trace_window.py $T --steps 10 --top 80 --out gpurun_out/${TAG}_window.txt > /dev/null
rm -f $T
