#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/bench_ab.sh "ENCDIFF_GEMM_XCD=0" "ENCDIFF_GEMM_XCD=2" "ENCDIFF_GEMM_XCD=0" "ENCDIFF_GEMM_XCD=2" || exit 1
ENCDIFF_GEMM_XCD=2 timeout -k 10 200 python tools/gemm_calls_time.py --out gpurun_out/calls_x2.json || exit 1
