"""Phase timing of the GroupNorm backward from in-kernel stamps (diagnostic library built with
-DED_GN_STAMP=1: python tools/build_variant.py gnstamp "norm.hip:-DED_GN_STAMP=1"):

    ENCDIFF_LIB=encdiff_amd/_ab/libencdiff_hip_gnstamp.so python tools/gn_stamps.py

Per shape (B=128, the step's levels): launch skew of block entries (realtime, 100 MHz), and per
block the shader cycles entry -> constants issued -> pass 1 done -> reduction done -> group terms
-> exit, averaged over blocks (median and max of the total).
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    from encdiff_amd import ops
    from encdiff_amd.ops import Geom
    lib = ops.lib
    B = 128
    for H, C_ in [(16, 64), (16, 128), (16, 192), (8, 256), (4, 512), (2, 256)]:
        g = Geom(B, H, H)
        x = torch.randn(g.pixels, C_, device="cuda").to(torch.bfloat16)
        y = torch.empty_like(x)
        gam = torch.ones(C_, device="cuda")
        bet = torch.zeros(C_, device="cuda")
        film = torch.randn(B, 2 * C_, device="cuda") * 0.1
        st = torch.empty(B * 32 * 2, device="cuda")
        dy = torch.randn_like(x)
        dx = torch.empty_like(x)
        rs = torch.randn_like(x)
        dgp = torch.empty(B, C_, device="cuda")
        dbp = torch.empty(B, C_, device="cuda")
        dfilm = torch.empty(B, 2 * C_, device="cuda")
        ops.groupnorm_fwd(x, g, gam, bet, y, st, 1e-5, True, film=film, ld_film=2 * C_)
        for _ in range(3):
            ops.groupnorm_bwd(x, g, gam, bet, st, 1e-5, True, dy, dx, dgp, dbp, film=film, ld_film=2 * C_,
                              dfilm=dfilm, ld_dfilm=2 * C_, resid=rs)
        torch.cuda.synchronize()
        cs = None
        nb = 16384
        buf = np.zeros((nb, 8), dtype=np.uint64)
        assert lib.encdiff_debug_gn_stamps(buf.ctypes.data_as(C.c_void_p), nb) == 0
        valid = buf[:, 0] > 0
        # the last launch's blocks: entries within 1 ms of the latest entry
        rt0 = buf[valid, 0].astype(np.int64)
        last = rt0 >= rt0.max() - 100000
        b = buf[valid][last].astype(np.int64)
        skew = (b[:, 0] - b[:, 0].min()) / 100.0  # us
        span = (b[:, 7].max() - b[:, 0].min()) / 100.0
        d = np.diff(b[:, 1:7], axis=1)
        tot = b[:, 6] - b[:, 1]
        print(f"H={H:2d} C={C_:3d} blocks={len(b):5d}  span {span:6.2f} us  entry skew max {skew.max():5.2f} us  "
              f"cycles: const {d[:, 0].mean():6.0f}  pass1 {d[:, 1].mean():6.0f}  reduce {d[:, 2].mean():6.0f}  "
              f"group {d[:, 3].mean():6.0f}  pass2 {d[:, 4].mean():6.0f}  total med {np.median(tot):6.0f} "
              f"max {tot.max():6.0f}", flush=True)


if __name__ == "__main__":
    main()
