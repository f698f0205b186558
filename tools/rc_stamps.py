"""Phase timing of encdiff_resconv_fwd from in-kernel stamps (diagnostic library built with
-DRC_STAMP=1: python tools/build_variant.py rcstamp "resconv.hip:-DRC_STAMP=1"):

    ENCDIFF_LIB=encdiff_amd/_ab/libencdiff_hip_rcstamp.so python tools/rc_stamps.py [--batch 8]

Per ResBlock conv shape of the Shapes3D UNet: the launch's span and entry skew (realtime, 100 MHz),
and per workgroup (wave 0) the shader cycles entry -> operands issued -> staged -> statistics ->
window normalised + B landed -> GEMM -> k-split combine -> exit, averaged over workgroups.
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--mask", type=int, default=0, help="EncdiffResConvArgs.skip_stages (stage ablation)")
    ap.add_argument("--waves", action="store_true", help="per-wave stamps (entry, issued, landed, at barrier)")
    a = ap.parse_args()
    from rc_bench import shapes
    from encdiff_amd import _lib as L
    from encdiff_amd import ops
    from encdiff_amd.ops import Geom
    lib = ops.lib
    lib.encdiff_debug_rc_stamps.argtypes = [C.c_void_p, C.c_int]
    if a.mask:
        fwd = L.lib.encdiff_resconv_fwd

        def masked(argp, s, _f=fwd):
            argp._obj.skip_stages = a.mask
            return _f(argp, s)
        L.lib.encdiff_resconv_fwd = masked
    dev, bf, B = "cuda", torch.bfloat16, a.batch
    names = ["issue", "stage", "stats", "norm+B", "gemm", "kred", "epi"]
    print(f"B={B}: cycles per phase (mean over workgroups): " + " ".join(names))
    for (h, cin, cout, rs, skip, film), n in sorted(shapes(B).items(), key=lambda kv: (-kv[0][0], kv[0][1])):
        ho = 2 * h if rs == 2 else (h // 2 if rs == 1 else h)
        x = (torch.randn(B * h * h, cin, device=dev) * 0.5).to(bf)
        w = (torch.randn(cout, 9 * cin, device=dev) * 0.02).to(bf)
        y = torch.empty(B * ho * ho, cout, device=dev, dtype=bf)
        gm, bt = torch.ones(cin, device=dev), torch.zeros(cin, device=dev)
        kw = dict(bias=torch.zeros(cout, device=dev))
        if film:
            kw.update(film=torch.zeros(B, 2 * cin, device=dev), ld_film=2 * cin)
        if skip.startswith("conv"):
            kw.update(xskip=(torch.randn(B * ho * ho, int(skip[4:]), device=dev)).to(bf))
            kw.update(wskip=torch.zeros(cout, kw["xskip"].shape[1], device=dev, dtype=bf), bskip=torch.zeros(cout, device=dev))
        elif skip.startswith("resid"):
            rr = int(skip[5:])
            hr = ho // 2 if rr == 2 else (ho * 2 if rr == 1 else ho)
            kw.update(resid=torch.zeros(B * hr * hr, cout, device=dev, dtype=bf), resid_resample=rr)
        for _ in range(3):
            assert ops.resconv_fwd(x, Geom(B, h, h), w, y, gm, bt, 1e-5, resample=rs, **kw)
        torch.cuda.synchronize()
        q = L.ResConvArgs(batch=B, h=h, cin=cin, cout=cout, resample=rs, groups=32, x=ops._p(x), ld_x=cin,
                          gamma=ops._p(gm), beta=ops._p(bt), w=ops._p(w), ld_w=9 * cin, y=ops._p(y), ld_y=cout)
        lds, grid = C.c_int(0), C.c_int(0)
        assert lib.encdiff_resconv_query(C.byref(q), C.byref(lds), C.byref(grid)) == 0
        nb = grid.value
        buf = np.zeros((4096, 10), dtype=np.uint64)
        assert lib.encdiff_debug_rc_stamps(buf.ctypes.data_as(C.c_void_p), 4096) == 0
        b = buf[:nb].astype(np.int64)
        skew = (b[:, 0] - b[:, 0].min()) / 100.0
        span = (b[:, 9].max() - b[:, 0].min()) / 100.0
        d = np.diff(b[:, 1:9], axis=1).mean(axis=0)
        print(f"h{h:<3} cin{cin:<4} cout{cout:<4} rs{rs} {skip:7s} grid {nb:4d} lds {lds.value // 1024:3d}K span {span:6.2f} us "
              f"skew {skew.max():5.2f} us | " + " ".join(f"{v:6.0f}" for v in d) + f" | total {d.sum():6.0f}", flush=True)
        if a.waves:  # per wave, relative to the workgroup's earliest wave entry: entry / issued / landed / at barrier
            fn = lib.encdiff_debug_rc_wstamps
            fn.argtypes = [C.c_void_p, C.c_int]
            wb = np.zeros((4096, 16, 4), dtype=np.uint64)
            assert fn(wb.ctypes.data_as(C.c_void_p), 4096) == 0
            w = wb[:nb, :8].astype(np.int64)
            rel = w - w[:, :, 0].min(axis=1)[:, None, None]
            m = rel.mean(axis=0)
            print("    per wave (entry, issued, landed, at barrier): " +
                  "  ".join(f"w{i}:{m[i, 0]:.0f}/{m[i, 1]:.0f}/{m[i, 2]:.0f}/{m[i, 3]:.0f}" for i in range(8)), flush=True)


if __name__ == "__main__":
    main()
