"""Time every recorded GEMM-family call of one eager training step (pairs, deferred finalizes and
weight-gradient grids as the step issues them), each replayed `reps` times inside a HIP graph.

    ENCDIFF_GEMM_XCD=0 python tools/gemm_calls_time.py --out gpurun_out/calls_x0.json

For A/B runs of a build-time or environment knob: diff two outputs call by call.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    import bench
    from encdiff_amd.trainer import HipTrainer
    torch.cuda.set_device(0)
    ldm, _ = bench.build_ldm()
    tr = HipTrainer(ldm, a.batch, graph=False)
    tr.init_scale_factor()
    tr.step_eager()
    calls = bench.record_gemms(tr)
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    out = []
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i, c in enumerate(calls):
            bench.replay_gemms([c])
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                bench.replay_gemms([c], reps=a.reps)
            g.replay()
            t0, t1 = ev(), ev()
            t0.record(s)
            g.replay()
            t1.record(s)
            s.synchronize()
            ps = [c[1]] if c[0] == "gemm" else ([c[1], c[2]] if c[0] == "pair_ex" else [c[1]])
            out.append({"i": i, "kind": c[0], "us": t0.elapsed_time(t1) / a.reps * 1e3,
                        "problems": [[p.M, p.N, p.K, p.a_mode, p.b_mode, p.c_mode, p.tile, p.split_k] for p in ps]})
    json.dump(out, open(a.out, "w"))
    print(f"{len(out)} calls, {sum(r['us'] for r in out):.1f} us total")


if __name__ == "__main__":
    main()
