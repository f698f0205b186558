#!/bin/bash
# round 4: LDM / DDIM tests, the default bench (DDIM + log_images legs), N=2 gloo DP rehearsal
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ldm.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ldm.log 2>&1 || { tail -30 gpurun_out/ldm.log; exit 1; }
tail -2 gpurun_out/ldm.log
timeout -k 10 400 python bench.py --skip-cpu --steps 30 > gpurun_out/b7.log 2>&1 || { tail -5 gpurun_out/b7.log; exit 1; }
tail -1 gpurun_out/b7.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['ddim_steps_per_sec'], d['ddim_steps_per_sec_b128'], d['ddim_log_images_s'])"
ENCDIFF_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --skip-cpu --skip-ddim > gpurun_out/r04_n2.log 2>&1 || { tail -20 gpurun_out/r04_n2.log; exit 1; }
grep '"metric"' gpurun_out/r04_n2.log | tail -1 > gpurun_out/r04_bench_n2_gloo_rehearsal.json
cut -c1-300 gpurun_out/r04_bench_n2_gloo_rehearsal.json
