"""GroupNorm forward / backward time per UNet shape (graph-timed) next to a plain copy of the
same bytes (the streaming floor), B=128.

    python tools/gn_bench.py
"""
from __future__ import annotations

import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def timed(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    from encdiff_amd import ops
    from encdiff_amd.ops import Geom
    L = ops.L
    B = 128
    shapes = [(16, 64), (16, 128), (16, 192), (8, 128), (8, 256), (8, 384), (4, 256), (4, 512), (2, 256), (2, 512)]
    for H, C in shapes:
        g = Geom(B, H, H)
        x = torch.randn(g.pixels, C, device="cuda").to(torch.bfloat16)
        y = torch.empty_like(x)
        gam = torch.ones(C, device="cuda")
        bet = torch.zeros(C, device="cuda")
        film = torch.randn(B, 2 * C, device="cuda") * 0.1
        st = torch.empty(B * 32 * 2, device="cuda")
        dy = torch.randn_like(x)
        dx = torch.empty_like(x)
        dgp = torch.empty(B, C, device="cuda")
        dbp = torch.empty(B, C, device="cuda")
        dfilm = torch.empty(B, 2 * C, device="cuda")
        fwd = lambda: ops.groupnorm_fwd(x, g, gam, bet, y, st, 1e-5, True, film=film, ld_film=2 * C)
        bwd = lambda: ops.groupnorm_bwd(x, g, gam, bet, st, 1e-5, True, dy, dx, dgp, dbp, film=film, ld_film=2 * C,
                                        dfilm=dfilm, ld_dfilm=2 * C)
        rs = torch.randn_like(x)
        bwr = lambda: ops.groupnorm_bwd(x, g, gam, bet, st, 1e-5, True, dy, dx, dgp, dbp, film=film, ld_film=2 * C,
                                        dfilm=dfilm, ld_dfilm=2 * C, resid=rs)
        cp = lambda: ops.ew(L.EW_COPY, x, y)
        tf, tb, tr, tc = timed(fwd), timed(bwd), timed(bwr), timed(cp)
        print(f"H={H:2d} C={C:3d} MB={x.numel() * 2 / 1e6:6.2f}  gn_fwd {tf:6.2f} us  gn_bwd {tb:6.2f} us  "
              f"+resid {tr:6.2f} us  copy {tc:6.2f} us", flush=True)


if __name__ == "__main__":
    main()
