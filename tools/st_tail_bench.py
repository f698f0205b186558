"""Time the fused SpatialTransformer tail kernel alone (graph of replays) at the sampling batch,
per level, with stages switched off through the debug mask (EncdiffStTailArgs.pad_: 1 no
cross-attention, 2 no feed-forward, 4 no LayerNorms, 8 16-row tiles) -- where the kernel's time goes.

    python tools/st_tail_bench.py [--batch 8]
"""
import argparse
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--eager", action="store_true", help="5 eager launches per case (PMC runs), no timing")
    ap.add_argument("--only", type=int, default=0, help="only this channel count")
    ap.add_argument("--head", action="store_true", help="head mode: stop after norm3 (t2, n3 written)")
    a = ap.parse_args()
    from encdiff_amd import _lib as L
    from encdiff_amd import ops
    dev = "cuda"
    bf = torch.bfloat16
    for c, hw in ((64, 256), (128, 64), (256, 16)):
        if a.only and c != a.only:
            continue
        rows = a.batch * hw
        r = lambda *s: (torch.randn(*s, device=dev) * 0.5).to(bf)  # noqa: E731
        o1, t0, x, out = r(rows, c), r(rows, c), r(rows, c), torch.empty(rows, c, device=dev, dtype=bf)
        kv = r(a.batch * 20, 2 * c)
        w = dict(out1=r(c, c), q2=r(c, c), out2=r(c, c), ff1=r(8 * c, c), ff2=r(c, 4 * c), po=r(c, c))
        for k in ("b_out1", "b_out2", "b_ff1", "b_ff2", "b_po", "be2", "be3"):
            w[k] = torch.zeros(8 * c if k == "b_ff1" else c, device=dev)
        w["g2"] = torch.ones(c, device=dev)
        w["g3"] = torch.ones(c, device=dev)
        head = (torch.empty(rows, c, device=dev, dtype=bf), torch.empty(rows, c, device=dev, dtype=bf)) if a.head else None
        for dbg in ((0,) if a.eager else (0, 1, 2, 4, 7, 8, 15)):
            orig = L.lib.encdiff_st_tail_fwd

            def f(argp, s, dbg=dbg):
                argp._obj.pad_ = dbg
                return orig(argp, s)
            L.lib.encdiff_st_tail_fwd = f
            try:
                run = lambda: ops.st_tail_fwd(o1, t0, x, kv[:, :c], kv[:, c:], w, out, rows, c, hw, 8, 20, 1e-5,  # noqa
                                                 head=head)
                run()
                if a.eager:
                    for _ in range(5):
                        run()
                    torch.cuda.synchronize()
                    continue
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(a.reps):
                        run()
                g.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                print(f"c={c:3d} rows={rows:5d} dbg={dbg}: {e0.elapsed_time(e1) * 1e3 / a.reps:7.2f} us", flush=True)
            finally:
                L.lib.encdiff_st_tail_fwd = orig


if __name__ == "__main__":
    main()
