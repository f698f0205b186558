#!/bin/bash
# GPU-box routine: HBM traffic of the GEMM family from two rocprofv3 PMC passes (FETCH_SIZE,
# WRITE_SIZE), summarised into profiles/gemm_traffic.json (see tools/gemm_traffic.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFG=${CONFIG:-shapes3d}   # CONFIG=celeba128: configs[4] -> gpurun_out/gemm_traffic_celeba128.json
OUT=gemm_traffic.json; [ $CFG = shapes3d ] || OUT=gemm_traffic_$CFG.json
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_f -o run -- python3 $R/tools/gemm_traffic.py run --config $CFG > $R/gpurun_out/pmc_f.log 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_w -o run -- python3 $R/tools/gemm_traffic.py run --config $CFG > $R/gpurun_out/pmc_w.log 2>&1 || { echo "write pass failed"; exit 1; }
cd $R && python tools/gemm_traffic.py summarize gpurun_out/pmc_f gpurun_out/pmc_w --out gpurun_out/$OUT
