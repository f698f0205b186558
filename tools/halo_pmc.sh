#!/bin/bash
# SQ counters + kernel durations of single conv GEMMs (tools/gemm_one.py), one rocprofv3 pass per
# counter group.  usage: bash tools/halo_pmc.sh TAG "<gemm_one args>" ["<gemm_one args>" ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
i=0
for ARGS in "$@"; do
  i=$((i+1))
  D=$R/gpurun_out/${TAG}_$i
  timeout -k 5 60 python3 $R/tools/gemm_one.py $ARGS --reps 20 > $D.time.log 2>&1 || { tail -3 $D.time.log; exit 1; }
  tail -1 $D.time.log
  timeout -s KILL 60 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o run -- python3 $R/tools/gemm_one.py $ARGS --reps 2 > $D.kt.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT --output-format csv -d $D/p1 -o run -- python3 $R/tools/gemm_one.py $ARGS --reps 2 > $D.p1.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVES --output-format csv -d $D/p2 -o run -- python3 $R/tools/gemm_one.py $ARGS --reps 2 > $D.p2.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $D/p3 -o run -- python3 $R/tools/gemm_one.py $ARGS --reps 2 > $D.p3.log 2>&1 || exit 1
done
cd $R && python3 - "$TAG" <<'PY'
import csv, glob, collections, sys
tag = sys.argv[1]
for d in sorted(glob.glob(f"gpurun_out/{tag}_*/")):
    print("==", d)
    for fn in glob.glob(d + "kt/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            if "gemm" in r["Name"]:
                print(f'   kernel {r["Name"][:70]} avg {float(r["AverageNs"])/1e3:.2f} us x{r["Calls"]}')
    for p in ("p1", "p2", "p3"):
        for fn in glob.glob(d + p + "/**/*counter_collection.csv", recursive=True):
            agg = collections.defaultdict(list)
            for r in csv.DictReader(open(fn)):
                if "gemm" in r["Kernel_Name"]:
                    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
            for c, v in sorted(agg.items()):
                print(f"   {c:28s} {sum(v) / len(v):14.0f}")
PY
