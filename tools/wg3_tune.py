"""Tune the WG3-paired 3x3 conv backward of one B=128 step: for each conv shape, the input
gradient's tile (64x64 / 128x64 / halo 16, 17, 22) x the WG3 split (half, planned, double), timed
in the step's steady state (consecutive pairs: each weight gradient's finalize rides in the next
launch; timing each pair with its own finalize picked small splits that lost in the step); writes the winners as table entries
(gpurun_out/wg3_tune.json: dgrad plan keys -> [tile, 1, us, 0], "wg3,h,cin,cout,rs" -> split).

    python tools/wg3_tune.py
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.wg3_bench import SHAPES  # noqa: E402


def main():
    from encdiff_amd import ops
    from encdiff_amd.ops import Geom
    L = ops.L
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

    table = {}
    B = 128
    for h, cin, cout, rs in SHAPES:
        g = Geom(B, h, h)
        gs = Geom(B, h // 2, h // 2) if rs == 2 else g
        x = torch.randn(gs.pixels, cin, device="cuda").to(bf)
        dy = torch.randn(g.pixels, cout, device="cuda").to(bf)
        wf = (torch.randn(cout, 9 * cin, device="cuda") * 0.02).to(bf)
        dw = torch.zeros(cout, 9 * cin, device="cuda")
        db = torch.zeros(cout, device="cuda")
        dx = torch.empty(g.pixels, cin, device="cuda", dtype=bf)
        sp0 = ops.wg3_split(B, h, h, cout, cin, rs, cout, cin, L.OUT_F32_ACCUM)
        splits = sorted({s for s in (sp0 // 2, sp0, sp0 * 2) if s >= 1 and B % s == 0 and
                         ((B // s // (1 if h == 16 else 2)) * (h // (4 if h == 4 else 2))) % 4 == 0})
        tiles = [4, 2] + [t for t in (16, 17, 22) if ops.halo_fits(t, B, h, h, cout, 0)]
        base = None
        res = []
        for tile in tiles:
            for sp in splits:
                ops.FORCE_TILE, ops.WG3_SPLIT = tile, sp
                try:
                    t = timed(lambda: ops.conv3x3_bwd_cl(dy, g, wf, x, cin, dw, dx, db, resample=rs))
                    ops.flush()
                except Exception as e:  # a tile the pair does not cover
                    print("skip", tile, sp, e)
                    continue
                finally:
                    ops.FORCE_TILE, ops.WG3_SPLIT = 0, 0
                res.append((t, tile, sp))
        ops.FORCE_TILE, ops.WG3_SPLIT = 0, 0
        base = timed(lambda: ops.conv3x3_bwd_cl(dy, g, wf, x, cin, dw, dx, db, resample=rs))
        ops.flush()
        t, tile, sp = min(res)
        print(f"h={h:2d} cin={cin:3d} cout={cout:3d} rs={rs}: current {base:6.2f} us -> best {t:6.2f} us "
              f"(dgrad tile {tile}, WG3 split {sp})", flush=True)
        table[ops.plan_key(g.pixels, cin, 9 * cout, L.OPA_IM2COL, L.OPB_CONV_DGRAD, L.OUT_BF16)] = [tile, 1, t, 0]
        table[f"wg3,{h},{cin},{cout},{rs}"] = sp
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(table, open("gpurun_out/wg3_tune.json", "w"), indent=0)


if __name__ == "__main__":
    main()
