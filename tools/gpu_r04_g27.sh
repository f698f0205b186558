#!/bin/bash
# round 4: GroupNorm backward with register-cached rows -- op + model tests, timing, short bench
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/ops27.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/ops27.log | head -20; tail -30 gpurun_out/ops27.log; exit 1; }
tail -1 gpurun_out/ops27.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_ldm.py tests/test_gpu_trainer.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/unet27.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/unet27.log | head; tail -20 gpurun_out/unet27.log; exit 1; }
tail -1 gpurun_out/unet27.log
timeout -k 10 200 python -u tools/gn_bench.py > gpurun_out/gn_bench.txt 2>&1 || { tail -5 gpurun_out/gn_bench.txt; exit 1; }
grep H= gpurun_out/gn_bench.txt | cut -c1-80
timeout -k 10 400 python bench.py --skip-cpu --steps 30 > gpurun_out/b27.log 2>&1 || { tail -5 gpurun_out/b27.log; exit 1; }
tail -1 gpurun_out/b27.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['ddim_steps_per_sec']['value'], d['ddim_steps_per_sec_b128']['value'])"
