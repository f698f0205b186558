"""Micro-benchmarks of the HBM-bound kernels at the EncDiff B=128 shapes (HIP events).

    python tools/kbench.py [--only gn,ln,attn,gemm,ew,sconv]

Prints per-shape microseconds and effective GB/s (algorithmic bytes: each operand read
once, each output written once).
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=30):
    """GPU time per call: `reps` calls captured in one HIP graph (no host launch cost)."""
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(st)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="gn,ln,attn,gemm,ew")
    ap.add_argument("--batch", type=int, default=128)
    a = ap.parse_args()
    from encdiff_amd import ops
    from encdiff_amd.ops import Geom
    B, dev = a.batch, "cuda"
    only = a.only.split(",")
    bf = torch.bfloat16
    if "gn" in only:
        tot_f = tot_b = 0.0
        for C, H, film in [(64, 16, True), (128, 16, True), (192, 16, True), (128, 8, True), (256, 8, True),
                           (384, 8, True), (256, 4, True), (512, 4, True), (256, 2, True), (512, 2, True)]:
            g = Geom(B, H, H)
            x = torch.randn(g.pixels, C, device=dev).to(bf)
            y = torch.empty_like(x)
            dx = torch.empty_like(x)
            gamma = torch.ones(C, device=dev)
            beta = torch.zeros(C, device=dev)
            E = torch.randn(B, 2 * C, device=dev) * 0.1
            dE = torch.zeros_like(E)
            st = torch.empty(B, 32, 2, device=dev)
            dgp = torch.empty(B, C, device=dev)
            dbp = torch.empty(B, C, device=dev)
            tf = timed(lambda: ops.groupnorm_fwd(x, g, gamma, beta, y, st, 1e-5, True, film=E, ld_film=2 * C))
            tb = timed(lambda: ops.groupnorm_bwd(x, g, gamma, beta, st, 1e-5, True, x, dx, dgp, dbp, film=E,
                                                 ld_film=2 * C, dfilm=dE, ld_dfilm=2 * C))
            nb = x.numel() * 2
            tot_f += tf
            tot_b += tb
            print(f"gn C={C:3d} H={H:2d}  fwd {tf:7.1f} us {2 * nb / tf / 1e3:7.0f} GB/s   "
                  f"bwd {tb:7.1f} us {3 * nb / tb / 1e3:7.0f} GB/s")
        print(f"gn total fwd {tot_f:.1f} us bwd {tot_b:.1f} us (one call per shape)")
    if "ln" in only:
        for rows, C in [(B * 256, 64), (B * 64, 128), (B * 16, 256), (B * 4, 256)]:
            x = torch.randn(rows, C, device=dev).to(bf)
            y = torch.empty_like(x)
            st = torch.empty(rows, 2, device=dev)
            gamma = torch.ones(C, device=dev)
            beta = torch.zeros(C, device=dev)
            parts = ops.layernorm_parts(rows, C)
            dgp = torch.empty(parts, C, device=dev)
            dbp = torch.empty(parts, C, device=dev)
            tf = timed(lambda: ops.layernorm_fwd(x, gamma, beta, y, st))
            tb = timed(lambda: ops.layernorm_bwd(x, gamma, st, x, y, dgp, dbp))
            nb = x.numel() * 2
            print(f"ln rows={rows:6d} C={C:3d}  fwd {tf:7.1f} us {2 * nb / tf / 1e3:7.0f} GB/s   "
                  f"bwd {tb:7.1f} us {3 * nb / tb / 1e3:7.0f} GB/s")
    if "attn" in only:
        for S, dh, sk in [(256, 8, 256), (64, 16, 64), (16, 32, 16), (4, 32, 4), (256, 8, 20), (64, 16, 20)]:
            heads = 8
            C = heads * dh
            q = torch.randn(B * S, C, device=dev).to(bf)
            k = torch.randn(B * sk, C, device=dev).to(bf)
            v = torch.randn(B * sk, C, device=dev).to(bf)
            o = torch.empty_like(q)
            lse = torch.empty(B * heads, S, device=dev)
            dq = torch.empty_like(q)
            dk = torch.empty_like(k)
            dv = torch.empty_like(v)
            tf = timed(lambda: ops.attention_fwd(q, k, v, o, lse, B, heads, S, sk, dh))
            tb = timed(lambda: ops.attention_bwd(q, k, v, o, lse, q, dq, dk, dv, B, heads, S, sk, dh))
            fl = 4.0 * B * heads * S * sk * dh
            print(f"attn S={S:3d} sk={sk:3d} dh={dh:2d}  fwd {tf:7.1f} us {fl / tf / 1e6:6.1f} TF/s   "
                  f"bwd {tb:7.1f} us {2.5 * fl / tb / 1e6:6.1f} TF/s")

    if "gemm" in only:
        # small linear GEMMs of the SpatialTransformers (token-major, K = C)
        for M, N, K in [(B * 256, 64, 64), (B * 256, 192, 64), (B * 256, 512, 64), (B * 256, 64, 256),
                        (B * 64, 128, 128), (B * 16, 256, 256), (B * 4, 256, 256)]:
            x = torch.randn(M, K, device=dev).to(bf)
            w = torch.randn(N, K, device=dev).to(bf) * 0.05
            y = torch.empty(M, N, device=dev, dtype=bf)
            dw = torch.zeros(N, K, device=dev)
            tf = timed(lambda: ops.linear_fwd(x, w, y))
            tw = timed(lambda: ops.linear_wgrad(y, x, dw))
            fl = 2.0 * M * N * K
            nb = 2.0 * (M * K + M * N)
            print(f"lin M={M:6d} N={N:4d} K={K:4d}  fwd {tf:7.1f} us {fl / tf / 1e6:6.1f} TF/s {nb / tf / 1e3:6.0f} GB/s"
                  f"   wgrad {tw:7.1f} us {fl / tw / 1e6:6.1f} TF/s {nb / tw / 1e3:6.0f} GB/s")
    if "ew" in only:
        x = torch.randn(1024, 64, device=dev).to(bf)
        y = torch.empty_like(x)
        t1 = timed(lambda: ops.ew_copy(x, y) if hasattr(ops, "ew_copy") else y.copy_(x))
        z = torch.empty(1, device=dev)
        t0 = timed(lambda: z.zero_())
        print(f"tiny kernels: 64K-elem copy {t1:.2f} us, torch 1-elem zero_ {t0:.2f} us")

    if "sconv" in only:  # output conv cin -> 3 (UNet out at 16x16 / 64, VQ conv_out at 16x16 / 128)
        for cin in (64, 128):
            g = Geom(B, 16, 16)
            h = torch.randn(g.pixels, cin, device=dev).to(bf)
            w = torch.randn(3, cin, 3, 3, device=dev) * 0.05
            b = torch.randn(3, device=dev)
            out = torch.empty(B, 3, 16, 16, device=dev)
            dy = torch.randn(B, 3, 16, 16, device=dev)
            dh = torch.empty_like(h)
            tf = timed(lambda: ops.small_conv_out_fwd(h, g, w, b, out))
            td = timed(lambda: ops.small_conv_out_bwd(h, g, w, dy, dh, None, None))
            nb = 2.0 * g.pixels * cin + 4.0 * g.pixels * 3
            print(f"out conv cin={cin:4d} 16x16  fwd {tf:6.1f} us {nb / tf / 1e3:6.0f} GB/s   "
                  f"dgrad {td:6.1f} us {nb / td / 1e3:6.0f} GB/s")


if __name__ == "__main__":
    main()
