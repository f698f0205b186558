"""Time the fused SpatialTransformer backward kernels alone (graph of replays) at the training
batch, per level, with stages switched off through the debug mask (EncdiffStTailBwdArgs.pad_: 1 no
GEGLU math, 2 no (row, head) attention pass, 4 no (head, key) dK / dV pass, 8 no LayerNorm math,
16 no gradient stores) -- where the tail kernel's time goes; the head kernel
and the forward tail at the same shape for reference.

    python tools/st_bwd_bench.py [--batch 128] [--masks 0,1,2,4,8,16,32,63]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def timed(run, reps):
    run()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            run()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--masks", default="0,1,2,4,8,16,31")
    a = ap.parse_args()
    from encdiff_amd import _lib as L
    from encdiff_amd import ops
    dev, bf = "cuda", torch.bfloat16
    for c, hw in ((64, 256), (128, 64)):
        rows, B, nctx = a.batch * hw, a.batch, 20
        r = lambda *s: (torch.randn(*s, device=dev) * 0.3).to(bf)  # noqa: E731
        save = dict(f=r(rows, 8 * c), t2=r(rows, c), t1=r(rows, c), q2=r(rows, c), o2=r(rows, c),
                    s3=torch.rand(rows, 2, device=dev) + 0.5, s2=torch.rand(rows, 2, device=dev) + 0.5,
                    lse2=torch.rand(B * 8, hw, device=dev) + 2.0)
        wt = dict(po=r(c, c), ff2=r(4 * c, c), ff1=r(c, 8 * c), out2=r(c, c), q2=r(c, c), out1=r(c, c))
        out = {k: torch.empty(rows, c, device=dev, dtype=bf) for k in ("d_t3", "d_t2", "d_q2", "d_t1", "d_o1")}
        out["d_f"] = torch.empty(rows, 8 * c, device=dev, dtype=bf)
        pm = torch.zeros(rows // 32, 4 * c, device=dev)
        kv, dkv = r(B * nctx, 2 * c), torch.empty(B * nctx, 2 * c, device=dev, dtype=bf)
        kv_part = torch.empty(rows // 32 * nctx, 2 * c, device=dev)
        g = torch.ones(c, device=dev)
        dy = r(rows, c)
        for dbg in [int(x) for x in a.masks.split(",")]:
            orig = L.lib.encdiff_st_tail_bwd

            def f(argp, s, dbg=dbg):
                argp._obj.pad_ = dbg
                return orig(argp, s)
            L.lib.encdiff_st_tail_bwd = f
            try:
                us = timed(lambda: ops.st_tail_bwd(dy, save, wt, g, g, kv[:, :c], kv[:, c:], out, (pm[:, :c], pm[:, c:2 * c]),
                                                   (pm[:, 2 * c:3 * c], pm[:, 3 * c:]), dkv[:, :c], dkv[:, c:], rows, c,
                                                   hw, 8, nctx, kv_part=kv_part), a.reps)
            finally:
                L.lib.encdiff_st_tail_bwd = orig
            print(f"tail_bwd c={c:3d} rows={rows:6d} dbg={dbg:2d}: {us:7.2f} us", flush=True)
        dqkv, wqkv, win = r(rows, 3 * c), r(c, 3 * c), r(c, c)
        tpi = hw // ops.st_tail_bwd_tile(c, rows, hw)
        us = timed(lambda: ops.st_head_bwd(dqkv, out["d_t1"], save["t1"], save["s2"], g, wqkv, win, out["d_t2"],
                                           out["d_q2"], (pm[:, :c], pm[:, c:2 * c]), rows, c,
                                           kv=(kv_part, tpi, nctx, B, dkv[:, :c], dkv[:, c:]) if tpi > 1 else None),
                   a.reps)
        print(f"head_bwd c={c:3d} rows={rows:6d}: {us:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
