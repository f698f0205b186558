#!/bin/bash
# SQ / TA counters + kernel trace of any short python tool run -> per-kernel averages.
# usage: bash tools/pmc_cmd.sh TAG "<python script and args>" [kernel-name filter]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; CMD=$2; FILT=${3:-gemm}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_kt -o run -- python3 $R/$CMD > $R/gpurun_out/${TAG}_kt.log 2>&1 || { tail -5 $R/gpurun_out/${TAG}_kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT --output-format csv -d $R/gpurun_out/${TAG}_p1 -o run -- python3 $R/$CMD > $R/gpurun_out/${TAG}_p1.log 2>&1 || { tail -5 $R/gpurun_out/${TAG}_p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVES --output-format csv -d $R/gpurun_out/${TAG}_p2 -o run -- python3 $R/$CMD > $R/gpurun_out/${TAG}_p2.log 2>&1 || { tail -5 $R/gpurun_out/${TAG}_p2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUSY_avr GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/gpurun_out/${TAG}_p3 -o run -- python3 $R/$CMD > $R/gpurun_out/${TAG}_p3.log 2>&1 || { tail -5 $R/gpurun_out/${TAG}_p3.log; exit 1; }
cd $R && python3 - "$TAG" "$FILT" <<'PY'
import csv, glob, collections, sys
tag, filt = sys.argv[1], sys.argv[2]
for fn in glob.glob(f"gpurun_out/{tag}_kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        if filt in r["Name"]:
            print(f"trace {r['Name'][:90]:90s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.2f} us")
for d in ("p1", "p2", "p3"):
    for fn in glob.glob(f"gpurun_out/{tag}_{d}/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(fn)):
            if filt not in r["Kernel_Name"]:
                continue
            k = r["Kernel_Name"][:90] + " grid=" + r.get("Grid_Size", "?")
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, cs in agg.items():
            print(d, k)
            for c, v in sorted(cs.items()):
                print(f"   {c:28s} {sum(v) / len(v):14.0f}")
PY
