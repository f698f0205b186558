#!/bin/bash
# round-4 evidence: full default bench (cpu_baseline, DDIM, log_images), rocprofv3 kernel stats of
# the same command, eager kernel-trace window, GEMM-family HBM traffic (FETCH_SIZE / WRITE_SIZE passes)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/round_profile.sh ${TAG:-r04} || exit 1
bash tools/gpu_traffic.sh || exit 1
cp gpurun_out/gemm_traffic.json gpurun_out/${TAG:-r04}_gemm_traffic.json
python -c "import json; d=json.load(open('gpurun_out/gemm_traffic.json')); print('traffic/alg', d['traffic_over_alg'], 'launches', d['launches'])"
