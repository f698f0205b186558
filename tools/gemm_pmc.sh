#!/bin/bash
# SQ stall counters of single GEMM shapes (tools/gemm_sweep.py --eager) -> gpurun_out/pmc_sq*/
# usage: bash tools/gemm_pmc.sh "<gemm_sweep args>"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
ARGS=${1:-"--M 2048 --N 256 --K 2304 --tiles 4,5 --splits 1"}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT --output-format csv -d $R/gpurun_out/pmc_sq1 -o run -- python3 $R/tools/gemm_sweep.py --eager --reps 5 $ARGS > $R/gpurun_out/pmc_sq1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_INST_LEVEL_LDS SQ_INSTS_SMEM SQ_WAVES --output-format csv -d $R/gpurun_out/pmc_sq2 -o run -- python3 $R/tools/gemm_sweep.py --eager --reps 5 $ARGS > $R/gpurun_out/pmc_sq2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUSY_avr GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/gpurun_out/pmc_ta -o run -- python3 $R/tools/gemm_sweep.py --eager --reps 5 $ARGS > $R/gpurun_out/pmc_ta.log 2>&1 || exit 1
cd $R && python3 - <<'PY'
import csv, glob, collections
for d in ("pmc_sq1", "pmc_sq2", "pmc_ta"):
    for fn in glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(fn)):
            if "gemm" not in r["Kernel_Name"]:
                continue
            k = r["Kernel_Name"][:60] + " grid=" + r.get("Grid_Size", "?")
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, cs in agg.items():
            print(d, k)
            for c, v in sorted(cs.items()):
                print(f"   {c:28s} {sum(v) / len(v):14.0f}")
PY
