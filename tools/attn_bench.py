"""Attention forward / backward at the UNet's shapes (B=128), graph-timed, or eager
repetitions for rocprofv3 --pmc (--eager).

    python tools/attn_bench.py [--eager] [--only 8]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--only", type=int, default=0, help="head dim to run (0: all)")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shape", default="", help="sq,sk,heads,dh[,fp8]: one shape instead of the UNet's "
                    "(configs[4]'s level 0: 1024,1024,8,16)")
    a = ap.parse_args()
    from encdiff_amd import ops
    from gn_bench import timed
    B = 128
    # (tokens, keys, heads, head dim): self / cross attention of the three attention levels
    shapes = [(256, 256, 8, 8), (256, 20, 8, 8), (64, 64, 8, 16), (64, 20, 8, 16), (16, 16, 8, 32), (16, 20, 8, 32)]
    f8 = False
    if a.shape:
        v = [int(x) for x in a.shape.split(",")]
        shapes, f8 = [tuple(v[:4])], len(v) > 4 and bool(v[4])
    for sq, sk, h, dh in shapes:
        if a.only and dh != a.only:
            continue
        c = h * dh
        q = (torch.randn(B * sq, c, device="cuda")).to(torch.bfloat16)
        k = (torch.randn(B * sk, c, device="cuda")).to(torch.bfloat16)
        v = (torch.randn(B * sk, c, device="cuda")).to(torch.bfloat16)
        o = torch.empty_like(q)
        lse = torch.empty(B * h, sq, device="cuda")
        do = torch.randn_like(q)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        fwd = lambda: ops.attention_fwd(q, k, v, o, lse, B, h, sq, sk, dh, fp8=f8)
        bwd = lambda: ops.attention_bwd(q, k, v, o, lse, do, dq, dk, dv, B, h, sq, sk, dh, fp8=f8)
        fwd()
        if a.eager:
            for _ in range(a.reps):
                fwd()
                bwd()
            torch.cuda.synchronize()
            print(f"sq={sq} sk={sk} dh={dh} eager x{a.reps}", flush=True)
            continue
        print(f"sq={sq:3d} sk={sk:3d} h={h} dh={dh:2d}  fwd {timed(fwd):7.2f} us  bwd {timed(bwd):7.2f} us", flush=True)


if __name__ == "__main__":
    main()
