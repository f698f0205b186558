#!/bin/bash
# round 4: GroupNorm-in-staging inference (unet tests), LDM / DDIM tests, default bench, N=2 gloo rehearsal
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/attn_bench.txt 2>&1 || { tail -5 gpurun_out/attn_bench.txt; exit 1; }
grep "dh= 8" gpurun_out/attn_bench.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet.py -x -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/unet.log 2>&1 || { grep -E "rel|PASS|FAIL|Error|error|assert" gpurun_out/unet.log | tail -30; exit 1; }
grep -E "agn|passed|failed" gpurun_out/unet.log | tail -6
timeout -k 10 600 python -u -m pytest tests/test_gpu_ldm.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ldm.log 2>&1 || { tail -30 gpurun_out/ldm.log; exit 1; }
tail -2 gpurun_out/ldm.log
timeout -k 10 400 python bench.py --skip-cpu --steps 30 > gpurun_out/b8.log 2>&1 || { tail -5 gpurun_out/b8.log; exit 1; }
tail -1 gpurun_out/b8.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['ddim_steps_per_sec'], d['ddim_steps_per_sec_b128'], d['ddim_log_images_s'])"
ENCDIFF_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --skip-cpu --skip-ddim > gpurun_out/r04_n2.log 2>&1 || { tail -20 gpurun_out/r04_n2.log; exit 1; }
grep '"metric"' gpurun_out/r04_n2.log | tail -1 > gpurun_out/r04_bench_n2_gloo_rehearsal.json
cut -c1-300 gpurun_out/r04_bench_n2_gloo_rehearsal.json
