#!/bin/bash
# GPU-box DP rehearsal: split-backward unit test, then 2 gloo ranks sharing the card with the
# split on / off / on, then world size 1 twice (determinism baseline); element-wise diffs.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_unet.py -x -q -s --timeout 200 --timeout-method thread > gpurun_out/unet_split.log 2>&1 || { tail -30 gpurun_out/unet_split.log; exit 1; }
tail -1 gpurun_out/unet_split.log
run() {  # tag nproc split
  DP_CHECK_SAVE=/tmp/dp_$1.pt ENCDIFF_DP_SPLIT=$3 ENCDIFF_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $2 --master-addr 127.0.0.1 --master-port 2954$4 tools/dp_split_check.py > gpurun_out/dpsplit_$1.log 2>&1 || { tail -30 gpurun_out/dpsplit_$1.log; return 1; }
  grep "digest" gpurun_out/dpsplit_$1.log
}
run a 2 1 1 && run b 2 0 2 && run c 2 1 3 && run w1a 1 1 4 && run w1b 1 1 5 || exit 1
python - <<'PY'
import torch
d = {k: torch.load(f"/tmp/dp_{k}.pt", weights_only=True) for k in ("a", "b", "c", "w1a", "w1b")}
def cmp(x, y):
    m0, m1 = d[x]["master"].double(), d[y]["master"].double()
    print(f"{x} vs {y}: max|dparam| {float((m0 - m1).abs().max()):.3e}  rel-L2 {float((m0 - m1).norm() / m0.norm()):.3e}")
cmp("a", "b"); cmp("a", "c"); cmp("w1a", "w1b")
PY
