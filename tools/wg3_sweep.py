"""WG3 (3x3 weight gradient) parameter sweep: ring depth (tile 32 / 33) x split, per shape,
kernel + finalize graph-timed.   python tools/wg3_sweep.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.wg3_bench import SHAPES  # noqa: E402


def main():
    from encdiff_amd import ops
    from encdiff_amd.ops import Geom
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

    for h, cin, cout, rs in SHAPES:
        g = Geom(128, h, h)
        gs = Geom(128, h // 2, h // 2) if rs == 2 else g
        x = torch.randn(gs.pixels, cin, device="cuda").to(bf)
        dy = torch.randn(g.pixels, cout, device="cuda").to(bf)
        dw = torch.zeros(cout, 9 * cin, device="cuda")
        out = []
        for tile in (32, 33):
            ops.WG3_TILE = tile
            for sp in (2, 4, 8, 16, 32):
                ni = 1 if h == 16 else 2
                st = (128 // sp // ni) * (h // (4 if h == 4 else 2)) if 128 % (sp * ni) == 0 else 0
                if not st or st % (8 if tile == 33 else 4):
                    continue
                ops.WG3_SPLIT = sp
                t = timed(lambda: ops.conv3x3_wgrad_cl(dy, x, g, cin, dw, None, resample=rs))
                out.append(f"{tile}/{sp}:{t:.1f}")
        ops.WG3_SPLIT = 0
        ops.WG3_TILE = 32
        print(f"h={h} cin={cin} cout={cout} rs={rs}: " + " ".join(out), flush=True)


if __name__ == "__main__":
    main()
