set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "step_prologue or gather" --timeout 120 --timeout-method thread > gpurun_out/pro.log 2>&1 || { tail -30 gpurun_out/pro.log; exit 1; }
tail -2 gpurun_out/pro.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_unet.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tr.log 2>&1 || { tail -30 gpurun_out/tr.log; exit 1; }
tail -2 gpurun_out/tr.log
timeout -k 10 300 python -u tools/call_gap.py > gpurun_out/call_gap.txt 2>&1 || { tail -5 gpurun_out/call_gap.txt; exit 1; }
timeout -k 10 200 python -u tools/call_gap.py --batch 8 --ddim > gpurun_out/call_gap_ddim8.txt 2>&1 || { tail -5 gpurun_out/call_gap_ddim8.txt; exit 1; }
timeout -k 10 300 python bench.py --skip-cpu --steps 30 > gpurun_out/b6.log 2>&1 || { tail -5 gpurun_out/b6.log; exit 1; }
tail -1 gpurun_out/b6.log | cut -c1-300
