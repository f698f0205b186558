"""Where the non-GEMM time goes: every GroupNorm / LayerNorm / attention / elementwise / fused
transformer launch of one eager B=128 training step (or DDIM sampling step, --ddim), recorded with
its arguments, then timed ALONE (graph of --reps replays each) and listed grouped by signature with
the streaming floor (bytes / 6.3 TB/s) next to it.

    python tools/call_gap.py [--batch 128] [--only groupnorm_bwd] [--ddim]
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

STRUCT_CALLS = ("encdiff_groupnorm_fwd", "encdiff_groupnorm_bwd", "encdiff_layernorm_fwd", "encdiff_layernorm_bwd",
                "encdiff_attention_fwd", "encdiff_attention_bwd", "encdiff_elementwise", "encdiff_st_tail_fwd",
                "encdiff_st_head_fwd", "encdiff_batchnorm_fwd", "encdiff_batchnorm_bwd", "encdiff_small_conv_fwd",
                "encdiff_small_conv_bwd")


def _copy(struct_type, ptr):
    s = struct_type()
    C.memmove(C.byref(s), ptr, C.sizeof(struct_type))
    return s


def record(run, L, only=None):
    """Run `run()` with every struct-argument entry point wrapped; returns [(name, args, keep)]."""
    calls = []
    protos = {n: L._PROTOS[n][0]._type_ for n in STRUCT_CALLS}
    orig = {n: getattr(L.lib, n) for n in STRUCT_CALLS}

    def wrap(name):
        def f(argp, stream):
            if only is None or name in only:
                a = _copy(protos[name], argp)
                keep = []
                xf = getattr(a, "x_from", None) if name.startswith("encdiff_groupnorm") else (
                    getattr(a, "dy_from", None) if name.startswith("encdiff_layernorm") else None)
                if xf:  # deep-copy the deferred producer's GemmArgs (its struct may not outlive the step)
                    g = _copy(L.GemmArgs, xf)
                    keep.append(g)
                    if name.startswith("encdiff_groupnorm"):
                        a.x_from = C.addressof(g)
                    else:
                        a.dy_from = C.addressof(g)
                calls.append((name, a, keep))
            return orig[name](argp, stream)
        return f
    for n in STRUCT_CALLS:
        setattr(L.lib, n, wrap(n))
    try:
        run()
    finally:
        for n in STRUCT_CALLS:
            setattr(L.lib, n, orig[n])
    torch.cuda.synchronize()
    return calls


def signature(name, a):
    short = name.replace("encdiff_", "")
    if short.startswith("groupnorm"):
        src = "slab" if getattr(a, "x_from", None) else ("stats" if getattr(a, "in_stats", None) else "")
        return f"{short} B{a.batch} hw{a.hw} c{a.c} film{int(bool(a.film))} silu{a.silu} {src}", \
            a.batch * a.hw * a.c * (6 if short.endswith("bwd") else 4)
    if short.startswith("layernorm"):
        src = "slab" if getattr(a, "dy_from", None) else ""
        return f"{short} rows{a.rows} c{a.c} {src}", a.rows * a.c * (6 if short.endswith("bwd") else 4)
    if short.startswith("attention"):
        return f"{short} B{a.batch} h{a.heads} sq{a.sq} sk{a.sk} dh{a.dh}", \
            2 * a.batch * a.heads * (a.sq + 2 * a.sk) * a.dh * (2 if short.endswith("bwd") else 1)
    if short == "elementwise":
        return f"ew op{a.op} {a.rows}x{a.cols}", 4 * a.rows * a.cols
    if short.startswith("st_"):
        return f"{short} rows{a.rows} c{a.c}", 0
    return short, 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--ddim", action="store_true", help="one DDIM sampling step's UNet forward instead")
    args = ap.parse_args()
    import encdiff_amd  # noqa: F401
    from encdiff_amd import _lib as L
    import bench
    only = None if not args.only else {"encdiff_" + o for o in args.only}
    ldm, _ = bench.build_ldm("shapes3d")
    if args.ddim:
        unet = ldm.model.diffusion_model
        x = torch.randn(args.batch, 3, 16, 16, device="cuda")
        t = torch.full((args.batch,), 500, device="cuda", dtype=torch.long)
        c = torch.randn(args.batch, 320, device="cuda")

        def run():
            with torch.no_grad():
                unet(x, t, context=[c])
        run()
    else:
        from encdiff_amd.trainer import HipTrainer
        tr = HipTrainer(ldm, args.batch, graph=False)
        tr.init_scale_factor()
        tr.step_eager()
        run = tr.step_eager
    torch.cuda.synchronize()
    calls = record(run, L, only)
    fns = {n: getattr(L.lib, n) for n in STRUCT_CALLS}

    def timeit(name, a):
        gs = torch.cuda.Stream()
        gs.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=gs):
            st = C.c_void_p(gs.cuda_stream)
            for _ in range(args.reps):
                L.check(fns[name](C.byref(a), st), name)
        g.replay()
        torch.cuda.synchronize()
        s, f = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        f.record()
        torch.cuda.synchronize()
        return s.elapsed_time(f) / args.reps * 1e3

    groups = defaultdict(lambda: [0, 0.0, 0.0])
    tot = defaultdict(float)
    for name, a, _keep in calls:
        t = timeit(name, a)
        key, by = signature(name, a)
        g = groups[key]
        g[0] += 1
        g[1] += t
        g[2] += by / 6.3e12 * 1e6
        tot[name.replace("encdiff_", "")] += t
    print(f"{len(calls)} calls; standalone ms per family: " +
          ", ".join(f"{k} {v / 1e3:.3f}" for k, v in sorted(tot.items(), key=lambda kv: -kv[1])))
    print(f"{'n':>3} {'us/call':>8} {'floor':>6} {'ms':>6}  signature")
    for k, (n, t, fl) in sorted(groups.items(), key=lambda kv: -kv[1][1]):
        print(f"{n:3d} {t / n:8.2f} {fl / n:6.2f} {t / 1e3:6.3f}  {k}")


if __name__ == "__main__":
    main()
