#!/bin/bash
# SQ counters of the fused transformer tail at the sampling batch (tools/st_tail_bench.py --eager)
#   bash tools/tail_pmc.sh [C=128] [BATCH=8]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
C=${1:-128}
B=${2:-8}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/tpmc1 -o run -- python3 $R/tools/st_tail_bench.py --eager --only $C --batch $B > $R/gpurun_out/tpmc1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SMEM --output-format csv -d $R/gpurun_out/tpmc2 -o run -- python3 $R/tools/st_tail_bench.py --eager --only $C --batch $B > $R/gpurun_out/tpmc2.log 2>&1 || exit 1
cd $R && python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(float)
n = collections.Counter()
for d in ("tpmc1", "tpmc2"):
    for fn in glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            if "st_tail" not in r["Kernel_Name"]:
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]] += 1
for k in sorted(tot):
    print(f"{k:28s} {tot[k] / n[k]:14.1f}  (per dispatch, {n[k]} dispatches)")
PY
