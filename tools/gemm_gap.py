"""Where the GEMM family's time goes: every GEMM-family call of one B=128 training step, timed
alone as the step issues it (graph of 10 replays), against its floor
max(2MNK / 2.5 PF, algorithmic bytes / 6.3 TB/s, 2 us).  Prints the calls grouped by signature
(count, us/call, floor, TF/s) sorted by total time above the floor.

    python tools/gemm_gap.py [--batch 128] [--top 40]
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
import sys
from collections import defaultdict

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    import encdiff_amd  # noqa: F401
    from encdiff_amd import _lib as L
    from encdiff_amd.trainer import HipTrainer
    import bench

    ldm, _ = bench.build_ldm("shapes3d")
    tr = HipTrainer(ldm, args.batch, graph=False)
    tr.init_scale_factor()
    tr.step_eager()
    torch.cuda.synchronize()
    recs = bench.record_gemms(tr)
    fns = {"gemm": L.lib.encdiff_gemm, "pair_ex": L.lib.encdiff_gemm_pair_ex,
           "finalize": L.lib.encdiff_gemm_finalize}

    def issue(rec, st):
        if rec[0] == "gemm":
            return fns["gemm"](C.byref(rec[1]), st)
        if rec[0] == "finalize":
            return fns["finalize"](C.byref(rec[1]), st)
        prev = C.byref(rec[3]) if rec[3] is not None else None
        return fns["pair_ex"](C.byref(rec[1]), C.byref(rec[2]), prev, rec[4], st)

    def timeit(rec):
        gs = torch.cuda.Stream()
        gs.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=gs):
            st = C.c_void_p(gs.cuda_stream)
            for _ in range(args.reps):
                issue(rec, st)
        g.replay()
        torch.cuda.synchronize()
        s, f = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        f.record()
        torch.cuda.synchronize()
        return s.elapsed_time(f) / args.reps * 1e3

    def cat(a):
        return {(1, 0): "conv_fwd", (1, 2): "conv_dgrad", (2, 3): "conv_wgrad", (0, 0): "lin_fwd",
                (0, 1): "lin_dgrad", (2, 1): "lin_wgrad", (1, 4): "k4s2_dgrad"}.get((a.a_mode, a.b_mode),
                                                                                      str((a.a_mode, a.b_mode)))

    def sig(a):
        return f"{cat(a)} {a.M}x{a.N}x{a.K} r{a.conv.resample} t{a.tile}/s{a.split_k}"

    groups = defaultdict(lambda: [0, 0.0, 0.0, 0.0])
    tot = 0.0
    for rec in recs:
        t = timeit(rec)
        tot += t
        if rec[0] == "finalize":
            key, fl, by = "finalize", 0.0, 0.0
        elif rec[0] == "gemm":
            a = rec[1]
            key, fl, by = sig(a), 2.0 * a.M * a.N * a.K, bench.gemm_alg_bytes(a)
        else:
            w, d = rec[1], rec[2]
            key = "pair[" + sig(w) + " | " + sig(d) + "]"
            fl = 2.0 * (w.M * w.N * w.K + d.M * d.N * d.K)
            by = bench.gemm_alg_bytes(w) + bench.gemm_alg_bytes(d)
        floor = max(fl / 2.5e15, by / 6.3e12, 2e-6) * 1e6
        g = groups[key]
        g[0] += 1
        g[1] += t
        g[2] += floor
        g[3] += fl
    print(f"{len(recs)} calls, {tot / 1e3:.3f} ms standalone sum")
    rows = sorted(groups.items(), key=lambda kv: -(kv[1][1] - kv[1][2]))
    print(f"{'n':>3} {'us/call':>8} {'floor':>6} {'gap_ms':>7} {'TF/s':>6}  signature")
    for k, (n, t, fl, f) in rows[:args.top]:
        print(f"{n:3d} {t / n:8.1f} {fl / n:6.1f} {(t - fl) / 1e3:7.3f} {f / t / 1e6:6.0f}  {k}")
    bycat = defaultdict(lambda: [0, 0.0, 0.0])
    for k, (n, t, fl, f) in groups.items():
        c = k.split()[0].lstrip("pair[")
        bycat[c][0] += n
        bycat[c][1] += t
        bycat[c][2] += f
    for c, (n, t, f) in sorted(bycat.items(), key=lambda kv: -kv[1][1]):
        print(f"category {c:12s} calls {n:4d} {t / 1e3:7.3f} ms {f / max(t, 1e-9) / 1e6:6.0f} TF/s")


if __name__ == "__main__":
    main()
