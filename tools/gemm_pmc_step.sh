#!/bin/bash
# GPU-box routine: SQ + L2 counters of the GEMM family replay (tools/gemm_traffic.py run), two
# --pmc passes with kernel traces, summarised per kernel class next to the traffic of
# gpurun_out/gemm_traffic.json (run tools/gpu_traffic.sh first) -> gpurun_out/gemm_pmc.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_WAVES --output-format csv -d $R/gpurun_out/gpmc_a -o run -- python3 $R/tools/gemm_traffic.py run > $R/gpurun_out/gpmc_a.log 2>&1 || { echo "pass a failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT --output-format csv -d $R/gpurun_out/gpmc_b -o run -- python3 $R/tools/gemm_traffic.py run > $R/gpurun_out/gpmc_b.log 2>&1 || { echo "pass b failed"; exit 1; }
cd $R && python3 tools/gemm_traffic.py pmc gpurun_out/gpmc_a gpurun_out/gpmc_b gpurun_out/gemm_traffic.json --out gpurun_out/gemm_pmc.txt
