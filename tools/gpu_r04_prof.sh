#!/bin/bash
# Round-4 profiling routine: GEMM-family gap table (every GEMM call of one B=128 step timed alone),
# eager kernel-trace window (all kernels, incl. torch's), short bench.
# usage: bash tools/gpu_r04_prof.sh TAG "tests..." [gap|nogap]
set -o pipefail
TAG=${1:-r04}; FOCUS=${2:-}; GAP=${3:-gap}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
if [ -n "$FOCUS" ]; then
  timeout -k 10 600 python -u -m pytest $FOCUS -x -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_focus.log 2>&1
  rc=$?
  grep -E "rel|PASS|FAIL|Error|error|assert|passed|failed" gpurun_out/${TAG}_focus.log | tail -40
  [ $rc = 0 ] || exit 1
fi
if [ "$GAP" = gap ]; then
  timeout -k 10 400 python -u tools/gemm_gap.py --top 80 > gpurun_out/${TAG}_gemm_gap.txt 2>&1 || { tail -5 gpurun_out/${TAG}_gemm_gap.txt; exit 1; }
  head -3 gpurun_out/${TAG}_gemm_gap.txt
fi
timeout -k 10 400 python bench.py --skip-cpu --steps 30 > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${TAG}_win -o run -- python3 $R/bench.py --steps 10 --warmup 3 --skip-ddim --skip-cpu --no-graph > $R/gpurun_out/${TAG}_win.log 2>&1 || { echo "window run failed"; exit 1; }
cd $R
T=$(find gpurun_out/${TAG}_win -name "*kernel_trace.csv" | head -1)
python tools/trace_window.py $T --steps 10 --top 400 --out gpurun_out/${TAG}_window.txt | head -3
rm -f $T
