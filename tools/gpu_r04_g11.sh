#!/bin/bash
# round 4: ops tests touched by the ADVICE fixes + attention backward trims, attention timing, DDIM AGN A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)} && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "encoder_head or cross_attention or deferred_finalize or step_prologue or attention" --timeout 200 --timeout-method thread > gpurun_out/ops11.log 2>&1 || { tail -30 gpurun_out/ops11.log; exit 1; }
tail -2 gpurun_out/ops11.log
timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/attn_bench.txt 2>&1 || { tail -5 gpurun_out/attn_bench.txt; exit 1; }
grep "dh= 8" gpurun_out/attn_bench.txt
bash tools/ddim_env_ab.sh 8 100 "ENCDIFF_AGN=0" "ENCDIFF_AGN=1" "ENCDIFF_AGN_RES=0" "ENCDIFF_AGN_FOLD=0" "ENCDIFF_AGN=0" "ENCDIFF_AGN=1" "ENCDIFF_AGN_RES=0" "ENCDIFF_AGN_FOLD=0"
