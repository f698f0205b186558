"""Time the fused AdamW + EMA kernel alone (graph of replays) over the configs[1] parameter count,
next to a plain copy of the same bytes.   python tools/opt_bench.py [--n 38840000]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
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
    ap.add_argument("--n", type=int, default=38840000)
    a = ap.parse_args()
    from encdiff_amd import ops
    n = a.n // 4 * 4
    p, gr, m, v, ema = (torch.randn(n, device="cuda") for _ in range(5))
    mirror = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    hyper = torch.tensor(ops.adamw_hyper(1e-4, 10, ema_one_minus_decay=1e-4), device="cuda", dtype=torch.float32)
    us = timed(lambda: ops.adamw_ema(p, gr, m, v, hyper, ema=ema, ema_n=n, mirror=mirror))
    nbytes = n * (20 + 18)
    src = torch.empty(nbytes // 8, device="cuda")
    dst = torch.empty_like(src)
    cu = timed(lambda: dst.copy_(src))
    print(f"adamw_ema n={n}: {us:.1f} us = {nbytes / us / 1e6:.2f} TB/s; copy of the same bytes {cu:.1f} us")


if __name__ == "__main__":
    main()
