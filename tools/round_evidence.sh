#!/bin/bash
# A round's committed evidence on one box: round_profile.sh (full default bench with cpu_baseline and
# the DDIM legs, rocprofv3 kernel statistics of the same command, eager kernel-trace window) and the
# GEMM-family HBM traffic (gpu_traffic.sh: FETCH_SIZE / WRITE_SIZE passes), TAG=<name>.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/round_profile.sh ${TAG:-round} || exit 1
bash tools/gpu_traffic.sh || exit 1
cp gpurun_out/gemm_traffic.json gpurun_out/${TAG:-round}_gemm_traffic.json
python -c "import json; d=json.load(open('gpurun_out/gemm_traffic.json')); print('traffic/alg', d['traffic_over_alg'], 'launches', d['launches'])"
