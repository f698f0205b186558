#!/bin/bash
# SQ counters of the attention kernels at one head dim (tools/attn_bench.py --eager)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
DH=${1:-8}
SHAPE=${SHAPE:+--shape $SHAPE}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --output-format csv -d $R/gpurun_out/apmc1 -o run -- python3 $R/tools/attn_bench.py --eager --only $DH $SHAPE --reps 5 > $R/gpurun_out/apmc1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_INST_LEVEL_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU_TRANS_F32 --output-format csv -d $R/gpurun_out/apmc2 -o run -- python3 $R/tools/attn_bench.py --eager --only $DH $SHAPE --reps 5 > $R/gpurun_out/apmc2.log 2>&1 || exit 1
cd $R && python3 - <<'PY'
import csv, glob, collections
for d in ("apmc1", "apmc2"):
    for fn in glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(fn)):
            if "attn" not in r["Kernel_Name"]:
                continue
            k = r["Kernel_Name"][:48] + " grid=" + r.get("Grid_Size", "?")
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, cs in agg.items():
            print(d, k)
            for c, v in sorted(cs.items()):
                print(f"   {c:28s} {sum(v) / len(v):14.0f}")
PY
