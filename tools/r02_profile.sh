#!/bin/bash
# Round-2 profiling: eager kernel-trace window of the training step (bench.py, 10 steps) and
# kernel statistics of a DDIM B=8 S=50 run.  usage: bash tools/r02_profile.sh TAG
set -o pipefail
TAG=${1:-r02}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
bash $R/tools/prof_window.sh ${TAG}_train || exit 1
head -45 $R/gpurun_out/${TAG}_train_window.txt | cut -c1-160
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_ddim -o run -- python3 $R/tools/ddim_prof.py --batch 8 --steps 50 > $R/gpurun_out/${TAG}_ddim.log 2>&1 || { echo "ddim prof failed"; tail -5 $R/gpurun_out/${TAG}_ddim.log; exit 1; }
cd $R
tail -2 gpurun_out/${TAG}_ddim.log
S=$(find gpurun_out/${TAG}_ddim -name "*kernel_stats.csv" | head -1)
python - "$S" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
calls = sum(int(r["Calls"]) for r in rows)
print(f"ddim trace: {calls} kernels, {tot/1e6:.2f} ms total")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:8.3f} ms {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:7.2f} us  {r["Name"][:110]}')
PY
find gpurun_out/${TAG}_ddim -name "*kernel_trace.csv" -delete
