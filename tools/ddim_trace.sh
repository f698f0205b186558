#!/bin/bash
# Kernel trace of DDIM B=8 (S=50, one captured loop replayed): per-step kernel statistics.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/ddimtr -o run -- python3 $R/tools/ddim_prof.py --batch 8 --steps 50 > $R/gpurun_out/ddimtr.log 2>&1 || exit 1
cd $R
N=$(python - <<'PY'
import sqlite3, glob
c = sqlite3.connect(glob.glob("gpurun_out/ddimtr/*.db")[0])
print(c.execute("select count(*) from kernels where name like '%ddim_kernel%'").fetchone()[0])
PY
)
T=$(python - <<'PY'
import sqlite3, glob
c = sqlite3.connect(glob.glob("gpurun_out/ddimtr/*.db")[0])
n = c.execute("select count(*) from kernels").fetchone()[0]
d = c.execute("select count(*) from kernels where name like '%ddim_kernel%'").fetchone()[0]
print(n * 50 // d)
PY
)
python tools/rocpd_stats.py $(ls gpurun_out/ddimtr/*.db | head -1) --last $T --per 50 --top 40 | cut -c1-170
rm -rf gpurun_out/ddimtr
