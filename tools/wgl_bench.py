"""Linear backward pairs of one B=128 training step: weight gradient on the split-K GEMM vs the WGL
kernel (gemm.hip tile 36), each paired with its input gradient (graph-timed, finalize flushed).

    python tools/wgl_bench.py
"""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (tokens, out, in, calls per step) of the UNet's linear layers with a weight gradient
SHAPES = [(32768, 64, 64, 25), (8192, 128, 128, 25), (2048, 256, 256, 25), (32768, 512, 64, 5),
          (8192, 1024, 128, 5), (2048, 2048, 256, 5), (32768, 64, 256, 5), (8192, 128, 512, 5),
          (2048, 256, 1024, 5), (32768, 192, 64, 5), (8192, 384, 128, 5), (2048, 768, 256, 5)]


def main():
    from encdiff_amd import ops
    bf = torch.bfloat16

    def timed(fn, reps=20):
        fn()
        torch.cuda.synchronize()
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(st):
            with torch.cuda.graph(g, stream=st):
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

    tot = {0: 0.0, 1: 0.0}
    for T, cout, cin, n in SHAPES:
        dy = torch.randn(T, cout, device="cuda").to(bf)
        x = torch.randn(T, cin, device="cuda").to(bf)
        w = (torch.randn(cout, cin, device="cuda") * 0.05).to(bf)
        dw = torch.zeros(cout, cin, device="cuda")
        db = torch.zeros(cout, device="cuda")
        dx = torch.empty(T, cin, device="cuda", dtype=bf)
        res = {}
        for wgl in (0, 1):
            ops.WGL = wgl
            a = ops.linear_wgrad_args(dy, x, dw, db)
            tp = timed(lambda: (ops.linear_bwd(dy, w, x, dx, dw, db), ops.flush()))
            res[wgl] = (tp, a.tile, a.split_k)
            tot[wgl] += n * tp
        ops.WGL = 1
        print(f"T={T:6d} out={cout:4d} in={cin:4d} x{n:2d}: pair gemm {res[0][0]:6.2f} (tile {res[0][1]} split "
              f"{res[0][2]:3d}) WGL {res[1][0]:6.2f} (split {res[1][2]:3d})", flush=True)
    print(f"per step: gemm {tot[0]:.1f} us, WGL {tot[1]:.1f} us")


if __name__ == "__main__":
    main()
