#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
TAG=r04g bash tools/gpu_r04_suite.sh || exit 1
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --skip-cpu > gpurun_out/r04g_bench_short.log 2>&1 || { tail -5 gpurun_out/r04g_bench_short.log; exit 1; }
tail -1 gpurun_out/r04g_bench_short.log > gpurun_out/r04g_bench_short.json
python -c "import json; d=json.load(open('gpurun_out/r04g_bench_short.json')); print(d['ms_per_step'], d['value'], d['roofline']['frac'], d['ddim_steps_per_sec'])"
