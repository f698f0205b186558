"""Run one GEMM shape repeatedly (for rocprofv3 PMC / kernel-trace studies of the engine).

    python tools/gemm_one.py conv --M 32768 --N 64 --cin 64 --h 16 [--tile 4 --split 1 --reps 50]
    python tools/gemm_one.py lin  --M 32768 --N 512 --K 64
    python tools/gemm_one.py wgrad --M 64 --N 64 --K 32768 --split 128
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kind", choices=["conv", "lin", "wgrad", "cwgrad"])
    ap.add_argument("--M", type=int, default=32768)
    ap.add_argument("--N", type=int, default=64)
    ap.add_argument("--K", type=int, default=64)
    ap.add_argument("--cin", type=int, default=64)
    ap.add_argument("--h", type=int, default=16)
    ap.add_argument("--tile", type=int, default=0)
    ap.add_argument("--split", type=int, default=0)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    from encdiff_amd import _lib as L
    from encdiff_amd import ops
    from encdiff_amd.ops import Geom
    dev = "cuda"
    bf = torch.bfloat16
    kw = {}
    if a.tile:
        kw["tile"] = a.tile
    if a.split:
        kw["split_k"] = a.split
    if a.kind == "conv":
        B = a.M // (a.h * a.h)
        g = Geom(B, a.h, a.h)
        x = torch.randn(g.pixels, a.cin, device=dev).to(bf)
        w = (torch.randn(a.N, 9 * a.cin, device=dev) * 0.05).to(bf)
        y = torch.empty(g.pixels, a.N, device=dev, dtype=bf)
        flops = 2.0 * g.pixels * a.N * 9 * a.cin

        def run():
            ops.gemm(g.pixels, a.N, 9 * a.cin, x, a.cin, w, 9 * a.cin, y, a.N, a_mode=L.OPA_IM2COL,
                     conv=ops._conv_geom(g, a.cin, 0, x), **kw)
    elif a.kind == "lin":
        x = torch.randn(a.M, a.K, device=dev).to(bf)
        w = (torch.randn(a.N, a.K, device=dev) * 0.05).to(bf)
        y = torch.empty(a.M, a.N, device=dev, dtype=bf)
        flops = 2.0 * a.M * a.N * a.K

        def run():
            ops.gemm(a.M, a.N, a.K, x, a.K, w, a.K, y, a.N, **kw)
    elif a.kind == "cwgrad":  # conv 3x3 weight gradient: M = cout, N = 9 * cin, K = pixels
        B = a.K // (a.h * a.h)
        g = Geom(B, a.h, a.h)
        dy = torch.randn(g.pixels, a.M, device=dev).to(bf)
        x = torch.randn(g.pixels, a.cin, device=dev).to(bf)
        dw = torch.zeros(a.M, 9 * a.cin, device=dev)
        flops = 2.0 * a.M * 9 * a.cin * g.pixels

        def run():
            ops.gemm(a.M, 9 * a.cin, g.pixels, dy, a.M, x, a.cin, dw, 9 * a.cin, a_mode=L.OPA_ROWM,
                     b_mode=L.OPB_IM2COL, c_mode=L.OUT_F32_ACCUM, conv=ops._conv_geom(g, a.cin, 0, x), **kw)
            ops.flush()
    else:
        dy = torch.randn(a.K, a.M, device=dev).to(bf)
        x = torch.randn(a.K, a.N, device=dev).to(bf)
        dw = torch.zeros(a.M, a.N, device=dev)
        flops = 2.0 * a.M * a.N * a.K

        def run():
            ops.gemm(a.M, a.N, a.K, dy, a.M, x, a.N, dw, a.N, a_mode=L.OPA_ROWM, b_mode=L.OPB_ROWN,
                     c_mode=L.OUT_F32_ACCUM, **kw)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g_ = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g_, stream=st):
        for _ in range(a.reps):
            run()
    g_.replay()
    torch.cuda.synchronize()
    s.record()
    g_.replay()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / a.reps * 1e3
    print(f"{a.kind} M={a.M} N={a.N} K={a.K} cin={a.cin}: {us:.2f} us/launch, {flops / us / 1e6:.1f} TF/s")
    for _ in range(5):  # eager launches for kernel-trace / PMC (graph replays are not traced)
        run()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
