"""Encoder4 BatchNorm forward / backward per trunk shape (B=128), graph-timed, next to a copy
of the same bytes.

    python tools/bn_bench.py
"""
from __future__ import annotations

import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))


def main():
    import encdiff_amd._lib as L
    from encdiff_amd import ops
    from gn_bench import timed
    B, C = 128, 128
    for H in (32, 16, 8, 4):
        rows = B * H * H
        x = (torch.randn(rows, C, device="cuda") * 2 + 0.5).to(torch.bfloat16)
        gamma = torch.rand(C, device="cuda") + 0.5
        beta = torch.randn(C, device="cuda") * 0.2
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        y = torch.empty_like(x)
        mean, rstd = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
        part = torch.empty(L.lib.encdiff_batchnorm_partials_floats(rows, C), device="cuda")
        cnt = torch.zeros(1, device="cuda", dtype=torch.int32)
        dy = torch.randn_like(x)
        dx = torch.empty_like(x)
        dg, db = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
        a = L.BatchNormArgs(rows=rows, c=C, eps=1e-5, momentum=0.1, relu=1, x=x.data_ptr(), ldx=C,
                            gamma=gamma.data_ptr(), beta=beta.data_ptr(), y=y.data_ptr(), ldy=C,
                            mean=mean.data_ptr(), rstd=rstd.data_ptr(), running_mean=rm.data_ptr(),
                            running_var=rv.data_ptr(), partials=part.data_ptr(), counter=cnt.data_ptr())
        a.dy, a.lddy, a.dx, a.lddx, a.dgamma, a.dbeta = dy.data_ptr(), C, dx.data_ptr(), C, dg.data_ptr(), db.data_ptr()

        def fwd():
            L.check(L.lib.encdiff_batchnorm_fwd(ctypes.byref(a), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "fwd")

        def bwd():
            L.check(L.lib.encdiff_batchnorm_bwd(ctypes.byref(a), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "bwd")
        cp = lambda: ops.ew(L.EW_COPY, x, y)
        print(f"H={H:2d} rows={rows:6d} MB={x.numel() * 2 / 1e6:6.2f}  bn_fwd {timed(fwd):6.2f} us  "
              f"bn_bwd {timed(bwd):6.2f} us  copy {timed(cp):6.2f} us", flush=True)


if __name__ == "__main__":
    main()
