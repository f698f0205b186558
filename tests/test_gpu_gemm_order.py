"""The XCD-aware tile order (gemm.hip xcd_remap, ENCDIFF_GEMM_XCD) only changes WHICH workgroup
computes a tile, never the arithmetic of a tile: one eager training step (B=32, every GEMM form --
forward convs / linears, paired input / weight gradients, WG3 / WGL grids, split-K slabs and
their finalizes) must give bitwise the same gradient arena and updated weights with the order off
(0), on for the weight gradients (2, the default) and on for every GEMM (1)."""
import hashlib
import os
import subprocess
import sys

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import hashlib, sys, torch
sys.path.insert(0, sys.argv[1])
import bench
from encdiff_amd.trainer import HipTrainer
torch.cuda.set_device(0)
ldm, _ = bench.build_ldm()
tr = HipTrainer(ldm, 32, graph=False)
tr.init_scale_factor()
tr.step_eager()
torch.cuda.synchronize()
h = hashlib.sha256()
for t in (tr.arena.grad, tr.arena.master):
    h.update(t.detach().cpu().numpy().tobytes())
print("HASH", h.hexdigest(), float(tr.arena.grad.abs().sum()))
"""


@pytest.mark.gpu
def test_gemm_xcd_order_is_bitwise_neutral():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = {}
    for mode in ("0", "2", "1"):
        env = dict(os.environ, ENCDIFF_GEMM_XCD=mode)
        r = subprocess.run([sys.executable, "-c", SCRIPT, REPO], cwd=REPO, env=env, capture_output=True, text=True,
                           timeout=240)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("HASH")][-1]
        out[mode] = line.split()
    assert float(out["0"][2]) > 0.0  # the step produced gradients
    assert out["2"][1] == out["0"][1], (out["0"], out["2"])
    assert out["1"][1] == out["0"][1], (out["0"], out["1"])
