#!/bin/bash
# Graph-replay kernel sequence of one step per environment arm (rocprofv3 kernel trace of the bench,
# tools/step_sequence.py) -> gpurun_out/seq_<i>.txt.   usage: bash tools/seq_ab.sh "A=0" "A=1"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
i=0
for e in "$@"; do
  cd /tmp && export TMPDIR=/tmp
  rm -rf $R/gpurun_out/seq_prof_$i
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/seq_prof_$i -o run -- python3 $R/bench.py --steps 10 --warmup 3 --skip-ddim --skip-cpu --skip-ref-api > $R/gpurun_out/seq_$i.log 2>&1 || { echo "prof $e failed"; tail -5 $R/gpurun_out/seq_$i.log; exit 1; }
  cd $R
  T=$(find gpurun_out/seq_prof_$i -name "*kernel_trace.csv" | head -1)
  python tools/step_sequence.py $T --steps 10 --out gpurun_out/seq_$i.txt > /dev/null || exit 1
  echo "$e: $(head -3 gpurun_out/seq_$i.txt | tr '\n' ' ')"
  rm -rf gpurun_out/seq_prof_$i
  i=$((i+1))
done
