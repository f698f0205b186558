#!/bin/bash
# round 4: norm.hip at -ffp-contract=on -- GN_FIN bitwise diagnosis, GroupNorm tests + timing, UNet tests, short bench
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 200 python tools/gnfin_diag.py > gpurun_out/gnfin_default.txt 2>&1 || { tail -5 gpurun_out/gnfin_default.txt; exit 1; }
sed -n 2,5p gpurun_out/gnfin_default.txt
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/ops20.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/ops20.log | head -20; tail -30 gpurun_out/ops20.log; exit 1; }
tail -1 gpurun_out/ops20.log
timeout -k 10 200 python -u tools/gn_bench.py > gpurun_out/gn_bench.txt 2>&1 || { tail -5 gpurun_out/gn_bench.txt; exit 1; }
grep H= gpurun_out/gn_bench.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_ldm.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/unet20.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/unet20.log | head; tail -20 gpurun_out/unet20.log; exit 1; }
tail -1 gpurun_out/unet20.log
timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/attn_bench.txt 2>&1 || { tail -5 gpurun_out/attn_bench.txt; exit 1; }
grep sq= gpurun_out/attn_bench.txt
timeout -k 10 400 python bench.py --skip-cpu --steps 30 > gpurun_out/b20.log 2>&1 || { tail -5 gpurun_out/b20.log; exit 1; }
tail -1 gpurun_out/b20.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['ddim_steps_per_sec'], d['ddim_steps_per_sec_b128'], d.get('ddim_log_images_s'))"
