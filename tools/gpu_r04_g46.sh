#!/bin/bash
# XCD-aware GEMM tile order: GEMM parity tests, step A/B (ENCDIFF_GEMM_XCD=0 / 1), traffic with it on.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "gemm or conv or linear or pair" > gpurun_out/g46_tests.log 2>&1 || { tail -20 gpurun_out/g46_tests.log; exit 1; }
tail -2 gpurun_out/g46_tests.log
bash tools/bench_ab.sh "ENCDIFF_GEMM_XCD=0" "ENCDIFF_GEMM_XCD=1" "ENCDIFF_GEMM_XCD=0" "ENCDIFF_GEMM_XCD=1" || exit 1
bash tools/gpu_traffic.sh > gpurun_out/g46_traffic.log 2>&1 || { tail -5 gpurun_out/g46_traffic.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/gemm_traffic.json')); print('traffic/alg', d['traffic_over_alg'])"
