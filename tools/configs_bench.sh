#!/bin/bash
# The other BASELINE configs' bench lines: configs[3] large batch (512 images / GPU) and configs[4]
# (celeba128, builder-defined).  TAG=<name>: outputs gpurun_out/TAG_bench_b512_config3.json and
# gpurun_out/TAG_bench_celeba128_config4.json (extra env passes through, e.g. ENCDIFF_ATTN_FP8=1).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
T=${TAG:-cfg}
timeout -k 10 500 python bench.py --batch 512 --skip-cpu --skip-ref-api --skip-ddim --steps 10 --warmup 3 > gpurun_out/${T}_b512.log 2>&1 || { tail -5 gpurun_out/${T}_b512.log; exit 1; }
tail -1 gpurun_out/${T}_b512.log > gpurun_out/${T}_bench_b512_config3.json
cut -c1-200 gpurun_out/${T}_bench_b512_config3.json
timeout -k 10 600 python bench.py --config celeba128 --skip-cpu --skip-ref-api --steps 10 --warmup 3 > gpurun_out/${T}_c4.log 2>&1 || { tail -5 gpurun_out/${T}_c4.log; exit 1; }
tail -1 gpurun_out/${T}_c4.log > gpurun_out/${T}_bench_celeba128_config4.json
cut -c1-200 gpurun_out/${T}_bench_celeba128_config4.json
