#!/bin/bash
# round 4: GroupNorm backward with register-cached rows -- GN tests, bitwise GN_FIN, timing, phase stamps
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "groupnorm" --timeout 200 --timeout-method thread > gpurun_out/gn24.log 2>&1 || { tail -30 gpurun_out/gn24.log; exit 1; }
tail -1 gpurun_out/gn24.log
timeout -k 10 200 python tools/gnfin_diag.py > gpurun_out/gnfin_default.txt 2>&1 || { tail -5 gpurun_out/gnfin_default.txt; exit 1; }
sed -n 2,4p gpurun_out/gnfin_default.txt
timeout -k 10 200 python -u tools/gn_bench.py > gpurun_out/gn_bench.txt 2>&1 || { tail -5 gpurun_out/gn_bench.txt; exit 1; }
grep H= gpurun_out/gn_bench.txt | cut -c1-80
ENCDIFF_LIB=encdiff_amd/_ab/libencdiff_hip_gnstamp.so timeout -k 10 200 python tools/gn_stamps.py > gpurun_out/gn_stamps.txt 2>&1 || { tail -5 gpurun_out/gn_stamps.txt; exit 1; }
grep H= gpurun_out/gn_stamps.txt
