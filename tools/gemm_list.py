"""Time every GEMM of one EncDiff training step with its current (tile, split) and print
the list grouped by role with each launch's roofline floor.

    python tools/gemm_list.py [--batch 128]

floor = max(flops / P_bf16, algorithmic bytes / BW) with P_bf16 = 2.5 PFLOP/s and
BW = 6.3 TB/s (achievable HBM, MI355X_MICROARCH.md); the gap column is time / floor.
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
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import encdiff_amd  # noqa: F401
    from encdiff_amd import _lib as L
    from encdiff_amd.configs import model_config
    from encdiff_amd.ldm.util import instantiate_from_config
    from encdiff_amd.trainer import HipTrainer
    import bench

    torch.manual_seed(0)
    ldm = instantiate_from_config(model_config("shapes3d")).cuda()
    tr = HipTrainer(ldm, args.batch, graph=False)
    tr.init_scale_factor()
    tr.step_eager()
    calls = bench.gemm_problems(bench.record_gemms(tr))
    orig = L.lib.encdiff_gemm
    ev = lambda: torch.cuda.Event(enable_timing=True)

    def timeit(a):
        gs = torch.cuda.Stream()
        gs.wait_stream(torch.cuda.current_stream())
        st = C.c_void_p(gs.cuda_stream)
        with torch.cuda.stream(gs):
            orig(C.byref(a), st)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=gs):
                for _ in range(args.reps):
                    orig(C.byref(a), st)
            g.replay()
            gs.synchronize()
            s, f = ev(), ev()
            s.record(gs)
            g.replay()
            f.record(gs)
            gs.synchronize()
        return s.elapsed_time(f) / args.reps * 1e3

    def cat(a):
        return {(1, 0): "conv_fwd", (1, 2): "conv_dgrad", (2, 3): "conv_wgrad", (0, 0): "lin_fwd",
                (0, 1): "lin_dgrad", (2, 1): "lin_wgrad"}.get((a.a_mode, a.b_mode), str((a.a_mode, a.b_mode)))

    # time each problem on its own (its own split-K finalize included, never deferred)

    seen = {}
    groups = defaultdict(list)
    for a in calls:
        key = (a.a_mode, a.b_mode, a.c_mode, a.M, a.N, a.K, a.split_k, a.tile, a.conv.resample)
        if key not in seen:
            seen[key] = [a, 0, timeit(a)]
        seen[key][1] += 1
    tot = defaultdict(float)
    totf = defaultdict(float)
    for key, (a, n, us) in seen.items():
        fl = 2.0 * a.M * a.N * a.K
        by = bench.gemm_alg_bytes(a)
        floor = max(fl / 2.5e15, by / 6.3e12) * 1e6
        groups[cat(a)].append((n * us, n, us, floor, a, fl, by))
        tot[cat(a)] += n * us
        totf[cat(a)] += n * floor
    for k in sorted(groups, key=lambda k: -tot[k]):
        print(f"== {k}: {tot[k]:.1f} us/step (floor {totf[k]:.1f})")
        for s, n, us, floor, a, fl, by in sorted(groups[k], key=lambda r: -r[0]):
            print(f"  {n:3d}x M={a.M:6d} N={a.N:5d} K={a.K:6d} rs={a.conv.resample} split={a.split_k:3d} "
                  f"tile={a.tile} cmode={a.c_mode} {us:7.1f}us floor {floor:6.1f} gap {us / floor:5.1f} "
                  f"{fl / us / 1e6:6.0f}TF {by / us / 1e3:6.0f}GB/s")
    print(f"TOTAL {sum(tot.values()):.1f} us/step, floor {sum(totf.values()):.1f}")


if __name__ == "__main__":
    main()
