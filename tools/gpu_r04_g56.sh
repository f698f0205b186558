#!/bin/bash
# tune (im2col keys with geometry) -> merge -> step A/B -> the B=512 / config4 trainer tests on the merged table
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
bash tools/gpu_r04_g50.sh || exit 1
ENCDIFF_GEMM_TILES=$R/gpurun_out/gemm_tiles_merged.json timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_trainer.py -m gpu > gpurun_out/g56_trainer.log 2>&1 || { grep -E "FAIL|Error" gpurun_out/g56_trainer.log | head; exit 1; }
tail -1 gpurun_out/g56_trainer.log
