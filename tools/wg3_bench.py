"""Time the 3x3 conv weight gradients of one B=128 training step: the WG3 kernel (gemm.hip
tile 32) against the split-K GEMM form (the measured table's tile / split), each launch with
its finalize, and the paired backward (weight + input gradient) both ways.

    python tools/wg3_bench.py [--batch 128] [--reps 20]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (h, cin, cout, resample) of the Shapes3D UNet's 3x3 convs with a weight gradient
SHAPES = [(16, 64, 64, 0), (16, 128, 64, 0), (16, 192, 64, 0), (16, 128, 128, 2), (8, 128, 128, 0),
          (8, 64, 128, 0), (8, 192, 128, 0), (8, 256, 128, 0), (8, 384, 128, 0), (8, 256, 256, 2),
          (4, 128, 256, 0), (4, 256, 256, 0), (4, 384, 256, 0), (4, 512, 256, 0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--eager", default="", help="h,cin,cout,rs: plain launches of that shape only (rocprofv3)")
    a = ap.parse_args()
    from encdiff_amd import ops
    from encdiff_amd.ops import Geom
    bf = torch.bfloat16

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(st):
            with torch.cuda.graph(g, stream=st):
                for _ in range(a.reps):
                    fn()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps * 1e3

    if a.eager:
        h, cin, cout, rs = map(int, a.eager.split(","))
        g = Geom(a.batch, h, h)
        gs = Geom(a.batch, h // 2, h // 2) if rs == 2 else g
        x = torch.randn(gs.pixels, cin, device="cuda").to(bf)
        dy = torch.randn(g.pixels, cout, device="cuda").to(bf)
        dw = torch.zeros(cout, 9 * cin, device="cuda")
        for wg3 in (0, 1):
            ops.WG3 = wg3
            for _ in range(5):
                ops.conv3x3_wgrad_cl(dy, x, g, cin, dw, None, resample=rs)
            torch.cuda.synchronize()
        return
    tot, totp = {}, {}
    for h, cin, cout, rs in SHAPES:
        g = Geom(a.batch, h, h)
        gs = Geom(a.batch, h // 2, h // 2) if rs == 2 else g
        x = torch.randn(gs.pixels, cin, device="cuda").to(bf)
        dy = torch.randn(g.pixels, cout, device="cuda").to(bf)
        wf = (torch.randn(cout, 9 * cin, device="cuda") * 0.02).to(bf)
        dw = torch.zeros(cout, 9 * cin, device="cuda")
        db = torch.zeros(cout, device="cuda")
        dx = torch.empty(g.pixels, cin, device="cuda", dtype=bf)
        flops = 2.0 * cout * 9 * cin * g.pixels
        res = {}
        for mode in ("gemm", 32, 34):
            ops.WG3 = mode != "gemm"
            ops.WG3_TILE = 32 if mode == "gemm" else mode
            args = ops.conv3x3_wgrad_cl_args(dy, x, g, cin, dw, db, rs)
            t = timed(lambda: ops.conv3x3_wgrad_cl(dy, x, g, cin, dw, db, resample=rs))
            tp = timed(lambda: (ops.conv3x3_bwd_cl(dy, g, wf, x, cin, dw, dx, db, resample=rs), ops.flush()))
            res[mode] = (t, tp, args.tile, args.split_k)
            tot[mode] = tot.get(mode, 0.0) + t
            totp[mode] = totp.get(mode, 0.0) + tp
        ops.WG3, ops.WG3_TILE = 1, 32
        print(f"h={h:2d} cin={cin:3d} cout={cout:3d} rs={rs}: wgrad gemm {res['gemm'][0]:6.2f} (split {res['gemm'][3]:3d}) "
              f"WG3 {res[32][0]:6.2f} (split {res[32][3]:3d}) | pair gemm {res['gemm'][1]:6.2f} WG3-paired "
              f"{res[32][1]:6.2f} WG3-serial {res[34][1]:6.2f} us", flush=True)
    print("sum wgrad: " + " ".join(f"{k}={v:.1f}" for k, v in tot.items()) + " | pairs: " +
          " ".join(f"{k}={v:.1f}" for k, v in totp.items()))


if __name__ == "__main__":
    main()
