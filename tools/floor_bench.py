"""Per-launch floors in graph replay: a 1-workgroup GEMM, small GEMMs of the DDIM B=8 shapes, a
tiny elementwise copy and an empty torch kernel (launch + dependent boundary), for the latency
budget of the small-batch (sampling) step.

    python tools/floor_bench.py
"""
from __future__ import annotations

import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))


def main():
    from encdiff_amd import ops
    from gn_bench import timed
    L = ops.L
    bf = torch.bfloat16
    dev = "cuda"
    x = torch.randn(64, 64, device=dev).to(bf)
    y = torch.empty_like(x)
    print(f"ew copy 4K elems          {timed(lambda: ops.ew(L.EW_COPY, x, y)):6.2f} us")
    t = torch.zeros(1, device=dev)
    print(f"torch add_ 1 elem         {timed(lambda: t.add_(1)):6.2f} us")
    for M, N, K, split in [(64, 64, 64, 1), (512, 64, 64, 1), (2048, 64, 64, 1), (2048, 64, 576, 1),
                           (128, 256, 2304, 8), (32, 256, 2304, 8), (32, 256, 2304, 1), (512, 128, 1152, 2)]:
        a = torch.randn(M, K, device=dev).to(bf)
        w = torch.randn(N, K, device=dev).to(bf) * 0.05
        o = torch.empty(M, N, device=dev, dtype=bf)
        us = timed(lambda: ops.gemm(M, N, K, a, K, w, K, o, N, split_k=split, tile=4))
        print(f"gemm {M:5d}x{N:4d}x{K:5d} split {split}: {us:6.2f} us")


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def boundary():
    """Per-node cost of a trivial kernel after producers of different sizes (graph replay): the
    dependent-boundary price inside a step (MI355X_MICROARCH.md price list 'boundary')."""
    from encdiff_amd import ops
    from gn_bench import timed
    L = ops.L
    bf = torch.bfloat16
    dev = "cuda"
    x = torch.randn(64, 64, device=dev).to(bf)
    y = torch.empty_like(x)
    ew = lambda: ops.ew(L.EW_COPY, x, y)  # noqa: E731
    print(f"ew alone                  {timed(ew):6.2f} us")
    for mb in (1, 4, 16):
        n = mb * 1024 * 1024 // 2
        a = torch.randn(n // 64, 64, device=dev).to(bf)
        b = torch.empty_like(a)
        big = lambda: ops.ew(L.EW_COPY, a, b)  # noqa: E731
        t_big = timed(big)
        t_pair = timed(lambda: (big(), ew()))
        print(f"copy {mb:2d} MB {t_big:6.2f} us; + trivial kernel after it: +{t_pair - t_big:5.2f} us")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "boundary":
    boundary()


def graph_size():
    """Per-node cost of trivial kernels vs the number of nodes in one captured graph, and with
    several distinct kernels interleaved (the step's graph holds ~840 nodes)."""
    from encdiff_amd import ops
    from gn_bench import timed
    L = ops.L
    bf = torch.bfloat16
    dev = "cuda"
    x = torch.randn(64, 64, device=dev).to(bf)
    y = torch.empty_like(x)
    t = torch.zeros(128, dtype=torch.long, device=dev)
    te = torch.empty(128, 64, device=dev, dtype=bf)
    z = torch.zeros(4096, device=dev)
    for reps in (50, 200, 800):
        print(f"{reps:4d} ew nodes: {timed(lambda: ops.ew(L.EW_COPY, x, y), reps=reps):6.2f} us/node; "
              f"ew+temb+torch add: {timed(lambda: (ops.ew(L.EW_COPY, x, y), ops.timestep_embedding(t, 64, te), z.add_(1)), reps=reps) / 3:6.2f} us/node",
              flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "graph":
    graph_size()


def after_real():
    """Marginal graph-replay cost of a trivial kernel placed after real step kernels (a conv GEMM,
    a GroupNorm), vs alone: does the dependent boundary grow behind real producers?"""
    from encdiff_amd import ops
    from encdiff_amd.ops import Geom
    from gn_bench import timed
    L = ops.L
    bf = torch.bfloat16
    dev = "cuda"
    x = torch.randn(64, 64, device=dev).to(bf)
    y = torch.empty_like(x)
    ew = lambda: ops.ew(L.EW_COPY, x, y)  # noqa: E731
    g = Geom(128, 16, 16)
    a = torch.randn(g.pixels, 64, device=dev).to(bf)
    w = (torch.randn(64, 576, device=dev) * 0.05).to(bf)
    o = torch.empty(g.pixels, 64, device=dev, dtype=bf)
    conv = lambda: ops.conv3x3_fwd(a, g, 64, w, o)  # noqa: E731
    gam, bet = torch.ones(64, device=dev), torch.zeros(64, device=dev)
    st = torch.empty(128, 64, device=dev)
    gn = lambda: ops.groupnorm_fwd(o, g, gam, bet, a, st, 1e-5, True)  # noqa: E731
    t_ew, t_conv, t_gn = timed(ew), timed(conv), timed(gn)
    print(f"ew {t_ew:6.2f}  conv {t_conv:6.2f}  gn {t_gn:6.2f} us")
    print(f"conv+ew {timed(lambda: (conv(), ew())):6.2f} (sum {t_conv + t_ew:6.2f})")
    print(f"conv+gn {timed(lambda: (conv(), gn())):6.2f} (sum {t_conv + t_gn:6.2f})")
    print(f"conv+gn+ew {timed(lambda: (conv(), gn(), ew())):6.2f}")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "real":
    after_real()
