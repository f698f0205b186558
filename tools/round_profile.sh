#!/bin/bash
# GPU-box routine for a round's committed evidence: full default bench (cpu_baseline, DDIM),
# rocprofv3 kernel statistics of the bench command, eager kernel-trace window of 10 steps.
# usage: bash tools/round_profile.sh TAG      (outputs under gpurun_out/TAG_*)
set -o pipefail
TAG=${1:-round}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 500 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_bench.json
cut -c1-200 gpurun_out/${TAG}_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_stats -o run -- python3 $R/bench.py --skip-cpu > $R/gpurun_out/${TAG}_stats.log 2>&1 || { echo "stats run failed"; exit 1; }
tail -1 $R/gpurun_out/${TAG}_stats.log | cut -c1-200
find $R/gpurun_out/${TAG}_stats -name "*kernel_trace.csv" -delete
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_win -o run -- python3 $R/bench.py --steps 10 --warmup 3 --skip-ddim --skip-cpu --skip-ref-api --no-graph > $R/gpurun_out/${TAG}_win.log 2>&1 || { echo "window run failed"; exit 1; }
cd $R
T=$(find gpurun_out/${TAG}_win -name "*kernel_trace.csv" | head -1)
python tools/trace_window.py $T --steps 10 --top 60 --out gpurun_out/${TAG}_window.txt | head -3
rm -f $T
