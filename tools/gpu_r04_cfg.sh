#!/bin/bash
# round 4: the other BASELINE configs' bench lines -- configs[3] large batch (512 / GPU), configs[4] celeba128
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 500 python bench.py --batch 512 --skip-cpu --skip-ddim --steps 10 --warmup 3 > gpurun_out/r04_b512.log 2>&1 || { tail -5 gpurun_out/r04_b512.log; exit 1; }
tail -1 gpurun_out/r04_b512.log > gpurun_out/r04_bench_b512_config3.json
cut -c1-200 gpurun_out/r04_bench_b512_config3.json
timeout -k 10 600 python bench.py --config celeba128 --skip-cpu --steps 10 --warmup 3 > gpurun_out/r04_c4.log 2>&1 || { tail -5 gpurun_out/r04_c4.log; exit 1; }
tail -1 gpurun_out/r04_c4.log > gpurun_out/r04_bench_celeba128_config4.json
cut -c1-200 gpurun_out/r04_bench_celeba128_config4.json
