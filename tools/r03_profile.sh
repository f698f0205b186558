#!/bin/bash
# Round-3 profile: kernel trace of graph-replayed bench steps -> ordered step sequence + stats.
# usage: bash tools/r03_profile.sh TAG [bench args]
set -o pipefail
TAG=${1:-r03}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_tr -o run -- python3 $R/bench.py --steps 10 --warmup 3 --skip-cpu --skip-ddim "$@" > $R/gpurun_out/${TAG}_tr.log 2>&1 || { echo "trace run failed"; tail -5 $R/gpurun_out/${TAG}_tr.log; exit 1; }
cd $R
tail -1 gpurun_out/${TAG}_tr.log | cut -c1-300
T=$(find gpurun_out/${TAG}_tr -name "*kernel_trace.csv" | head -1)
python tools/step_sequence.py $T --steps 10 --out gpurun_out/${TAG}_sequence.txt
python tools/trace_window.py $T --steps 10 --top 70 --out gpurun_out/${TAG}_window.txt | head -2
rm -f $T
