#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
ENCDIFF_GEMM_XCD=0 timeout -k 10 200 python tools/gemm_calls_time.py --out gpurun_out/calls_x0.json || exit 1
ENCDIFF_GEMM_XCD=1 timeout -k 10 200 python tools/gemm_calls_time.py --out gpurun_out/calls_x1.json || exit 1
