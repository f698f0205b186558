"""K-sweep of one GEMM shape: graph-timed time per launch for each (tile, split, K), to split
a launch's time into a fixed part (launch, prologue, epilogue) and a per-k-tile part.

    python tools/gemm_sweep.py --M 2048 --N 256 --K 64,576,1152,2304,4608 --tiles 4,5 --splits 1,4
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=2048)
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--K", default="64,576,1152,2304,4608")
    ap.add_argument("--tiles", default="4,5")
    ap.add_argument("--splits", default="1,4")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--f32", action="store_true", help="fp32 output (no bf16 epilogue)")
    ap.add_argument("--eager", action="store_true", help="plain launches, no graph (for rocprofv3 --pmc)")
    a = ap.parse_args()
    from encdiff_amd import ops
    L = ops.L
    M, N = a.M, a.N
    for K in map(int, a.K.split(",")):
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
        out = torch.empty(M, N, device="cuda", dtype=torch.float32 if a.f32 else torch.bfloat16)
        cm = L.OUT_F32 if a.f32 else L.OUT_BF16
        for tile in map(int, a.tiles.split(",")):
            for split in map(int, a.splits.split(",")):
                if split > 1 and K // split < 64:
                    continue
                run = lambda: ops.gemm(M, N, K, x, K, w, K, out, N, c_mode=cm, split_k=split, tile=tile)
                run()
                torch.cuda.synchronize()
                if a.eager:
                    for _ in range(a.reps):
                        run()
                    torch.cuda.synchronize()
                    print(f"M={M} N={N} K={K} tile={tile} split={split} eager x{a.reps}", flush=True)
                    continue
                g = torch.cuda.CUDAGraph()
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    with torch.cuda.graph(g, stream=s):
                        for _ in range(a.reps):
                            run()
                g.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / a.reps * 1e3
                kt = -(-K // 64) // split
                print(f"M={M} N={N} K={K:6d} tile={tile} split={split:3d} ktiles/block={kt:4d} {us:8.2f} us "
                      f"{2.0 * M * N * K / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
