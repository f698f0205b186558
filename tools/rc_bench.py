"""Time encdiff_resconv_fwd alone (graph of back-to-back launches) for every distinct ResBlock conv
of the Shapes3D UNet at a sampling batch, with stages switched off through the debug mask
(EncdiffResConvArgs.skip_stages: 1 no staging loads, 2 no normalisation, 4 no GEMM, 8 no stores)
and with plan overrides -- where the kernel's time goes.

    python tools/rc_bench.py [--batch 8] [--masks 0,1,4] [--tiles 0:0,1:2]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def shapes(B):
    from encdiff_amd.ldm.modules.diffusionmodules.openaimodel_enc import UNetModel
    from encdiff_amd.unet import ResSpec
    from oracle import encdiff_oracle as O
    m = UNetModel(**O.SHAPES3D_UNET).cuda()
    sp = m.executor().spec
    out = {}
    for blk in sp.input_blocks + [sp.middle] + sp.output_blocks:
        for r in blk:
            if not isinstance(r, ResSpec):
                continue
            k1 = (r.hin, r.cin, r.cout, r.updown, "none", False)
            skip = ("conv%d" % r.cin) if r.cin != r.cout else ("resid%d" % r.updown)
            k2 = (r.hout, r.cout, r.cout, 0, skip, True)
            for k in (k1, k2):
                out[k] = out.get(k, 0) + 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--masks", default="0,1,2,4,8")
    ap.add_argument("--tiles", default="0:0")
    a = ap.parse_args()
    from encdiff_amd import _lib as L
    from encdiff_amd import ops
    from encdiff_amd.ops import Geom
    dev, bf = "cuda", torch.bfloat16
    B = a.batch
    masks = [int(v) for v in a.masks.split(",")]
    tiles = [tuple(int(u) for u in v.split(":")) for v in a.tiles.split(",")]
    tot = {}

    def graph_us(run):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(a.reps):
                run()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1000 / (5 * a.reps)
    src, dst = torch.zeros(64, 64, device=dev, dtype=bf), torch.zeros(64, 64, device=dev, dtype=bf)
    print(f"launch floor (a 64x64 elementwise copy, same graph form): {graph_us(lambda: ops.ew(L.EW_COPY, src, dst)):.2f} us")
    print(f"B={B}: us per launch (graph of {a.reps}); columns: skip_stages masks {masks} per tile override")
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
        row = []
        for tl in tiles:
            for mk in masks:
                orig = L.lib.encdiff_resconv_fwd

                def f(argp, s, mk=mk):
                    argp._obj.skip_stages = mk
                    return orig(argp, s)
                L.lib.encdiff_resconv_fwd = f
                ops.RC_TILE_M, ops.RC_TILE_N = tl
                try:
                    run = lambda: ops.resconv_fwd(x, Geom(B, h, h), w, y, gm, bt, 1e-5, resample=rs, **kw)  # noqa
                    try:
                        ok = run()
                    except Exception:  # a plan override this shape does not take
                        ok = False
                    if not ok:
                        row.append("  unsup")
                        continue
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        for _ in range(a.reps):
                            run()
                    g.replay()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(5):
                        g.replay()
                    e1.record()
                    torch.cuda.synchronize()
                    us = e0.elapsed_time(e1) * 1000 / (5 * a.reps)
                    row.append(f"{us:7.2f}")
                    tot[(tl, mk)] = tot.get((tl, mk), 0.0) + us * n
                finally:
                    L.lib.encdiff_resconv_fwd = orig
                    ops.RC_TILE_M, ops.RC_TILE_N = 0, 0
        print(f"h{h:<3} cin{cin:<4} cout{cout:<4} rs{rs} {skip:7s} x{n:<2}: " + " ".join(row), flush=True)
    print("per UNet forward (us): " + "  ".join(f"tiles{k[0]} mask{k[1]}: {v:.1f}" for k, v in tot.items()))


if __name__ == "__main__":
    main()
