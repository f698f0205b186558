#!/bin/bash
# GPU-box routine: gpu tests, bench (graph), eager kernel-trace window of the timed region.
# usage: bash tools/gpu_check.sh TAG [bench args...]
set -o pipefail
TAG=${1:-run}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -m pytest tests/ -q -m gpu -rf -x > gpurun_out/${TAG}_tests.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python bench.py --skip-cpu "$@" > gpurun_out/${TAG}_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --skip-ddim --skip-cpu --no-graph "$@" > $R/gpurun_out/${TAG}_prof.log 2>&1 || { echo "prof failed"; exit 1; }
cd $R
T=$(find gpurun_out/${TAG}_prof -name "*kernel_trace.csv" | head -1)
python tools/trace_window.py $T --steps 10 --top 60 --out gpurun_out/${TAG}_window.txt | head -30
rm -f $T
