#!/bin/bash
# round 4: explicit-FMA split-K combine (finalize / fold / norm slab combines), attention trims:
# op tests, UNet + LDM tests, attention timing, short bench
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/ops17.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/ops17.log | head -20; tail -30 gpurun_out/ops17.log; exit 1; }
tail -1 gpurun_out/ops17.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_ldm.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/unet17.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/unet17.log | head; tail -20 gpurun_out/unet17.log; exit 1; }
tail -1 gpurun_out/unet17.log
timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/attn_bench.txt 2>&1 || { tail -5 gpurun_out/attn_bench.txt; exit 1; }
grep sq= gpurun_out/attn_bench.txt
timeout -k 10 400 python bench.py --skip-cpu --steps 30 > gpurun_out/b17.log 2>&1 || { tail -5 gpurun_out/b17.log; exit 1; }
tail -1 gpurun_out/b17.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['ddim_steps_per_sec'], d['ddim_steps_per_sec_b128'], d.get('ddim_log_images_s'))"
