"""Record every GEMM of one EncDiff training step and time each under every tile shape.

    python tools/gemm_profile.py [--batch 128] [--write-table]

Prints per-category totals (current heuristic vs best tile) and, with --write-table,
stores the best tile per GEMM signature in encdiff_amd/gemm_tiles.json (read by
ops.gemm at run time).  Also prints a phase breakdown of the eager step (HIP events).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
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
    ap.add_argument("--pairs", type=int, default=1, help="choose paired wgrad/dgrad tiles by timing the pair")
    ap.add_argument("--wg", type=int, default=1, help="sweep the WG3 / WGL weight-gradient kernels' splits too")
    ap.add_argument("--write-table", default="", help="path for the measured (tile, split) table, e.g. "
                    "gpurun_out/gemm_tiles.json (copy it to encdiff_amd/gemm_tiles.json)")
    ap.add_argument("--only-h", default="", help="comma list of conv sizes h: sweep only the implicit-im2col "
                    "problems (and their pairs) at those sizes, keeping every other entry of the current table")
    args = ap.parse_args()
    import encdiff_amd  # noqa: F401
    from encdiff_amd import _lib as L
    from encdiff_amd import ops
    from encdiff_amd.configs import model_config
    from encdiff_amd.ldm.util import instantiate_from_config
    from encdiff_amd.trainer import HipTrainer

    torch.manual_seed(0)
    ldm = instantiate_from_config(model_config("shapes3d")).cuda()
    tr = HipTrainer(ldm, args.batch, graph=False)
    tr.init_scale_factor()
    tr.step_eager()
    torch.cuda.synchronize()

    # ---- phase breakdown (eager) --------------------------------------------------
    ev = lambda: torch.cuda.Event(enable_timing=True)
    e = [ev() for _ in range(8)]
    img = tr.img
    e[0].record()
    with torch.no_grad():
        z = ldm.get_first_stage_encoding(ldm.encode_first_stage(img))
    e[1].record()
    c = ldm.get_learned_conditioning(img)
    e[2].record()
    t = torch.randint(0, 1000, (args.batch,), device="cuda")
    noise = torch.randn_like(z)
    xn = ldm.q_sample(z, t, noise)
    unet = ldm.model.diffusion_model
    ex = unet.executor()
    eps = ex.forward(xn, t, c.detach())
    e[3].record()
    d_c = ex.backward(torch.sign(eps - noise) / eps.numel())
    e[4].record()
    c.backward(d_c)
    e[5].record()
    tr.opt.stage_hyper()
    tr.opt.launch()
    e[6].record()
    torch.cuda.synchronize()
    names = ["vq_encode", "encoder4_fwd", "unet_fwd(+q_sample)", "unet_bwd", "encoder4_bwd", "adamw+ema+pack"]
    for i, n in enumerate(names):
        print(f"phase {n:22s} {e[i].elapsed_time(e[i + 1]):8.3f} ms")

    # ---- record GEMMs (every problem of one training step, incl. the paired ones) ----
    import bench
    calls = bench.gemm_problems(bench.record_gemms(tr))
    print(f"{len(calls)} GEMM problems per training step")
    orig = L.lib.encdiff_gemm

    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)

    ws = ops._workspace()

    def timeit(a, tile, split=None, fold=False):
        a2 = L.GemmArgs()
        C.memmove(C.byref(a2), C.byref(a), C.sizeof(L.GemmArgs))
        a2.tile = tile
        if split is not None:
            a2.split_k = split
            a2.workspace = ws.data_ptr() if split > 1 else None
            a2.split_counters = (ops._counters().data_ptr() if split > 1 and fold and
                                 a2.a_mode != L.OPA_ROWM else None)
            if split > 1 and a2.c_mode in (L.OUT_BF16, L.OUT_F32, L.OUT_F32_ACCUM) and split * a2.M * (a2.N + 1) > ops.WS_FLOATS:
                return float("inf")
        for _ in range(2):
            rc = orig(C.byref(a2), stream)
            if rc != 0:
                return float("inf")
        # GPU time: the reps are captured in a graph (no host launch gaps)
        gs = torch.cuda.Stream()
        gs.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=gs):
            st = C.c_void_p(gs.cuda_stream)
            for _ in range(args.reps):
                orig(C.byref(a2), st)
        g.replay()
        torch.cuda.synchronize()
        s, f = ev(), ev()
        s.record()
        g.replay()
        f.record()
        torch.cuda.synchronize()
        return s.elapsed_time(f) / args.reps * 1e3

    def cat(a):
        modes = (a.a_mode, a.b_mode)
        return {(1, 0): "conv_fwd", (1, 2): "conv_dgrad", (2, 3): "conv_wgrad", (0, 0): "lin_fwd",
                (0, 1): "lin_dgrad", (2, 1): "lin_wgrad"}.get(modes, str(modes))

    def key_of(a):  # implicit-im2col problems keyed with their geometry (ops.plan_key)
        im2 = a.a_mode == L.OPA_IM2COL or a.b_mode == L.OPB_IM2COL
        return ops.plan_key(a.M, a.N, a.K, a.a_mode, a.b_mode, a.c_mode, a.conv.resample, a.conv.h if im2 else 0)

    only_h = {int(x) for x in args.only_h.split(",") if x}

    def selected(a):
        return not only_h or ((a.a_mode == L.OPA_IM2COL or a.b_mode == L.OPB_IM2COL) and a.conv.h in only_h)

    tot_cur, tot_best = defaultdict(float), defaultdict(float)
    flops = defaultdict(float)
    table = dict(ops._tile_table()) if only_h else {}
    rows = []
    done = {}
    for a in calls:
        key = key_of(a)
        if not selected(a):
            continue
        if key in done:  # same problem already swept: reuse
            cur, best_tile, best_split, best_t, best_fold = done[key]
            k = cat(a)
            tot_cur[k] += cur
            tot_best[k] += best_t
            flops[k] += 2.0 * a.M * a.N * a.K
            continue
        cur = timeit(a, a.tile)
        best_t, best_tile, best_split, best_fold = cur, a.tile, a.split_k, bool(a.split_counters)
        # weight gradients run inside the paired kernel (64 x 64 tiles, k stages 64 or 128) with their slabs in
        # one workspace half (deferred finalize): only splits that fit are candidates
        wgrad = a.a_mode == L.OPA_ROWM
        # input gradients run paired with their weight gradient: one grid sizes every workgroup's
        # LDS for the larger tile, so the deep-ring / deep-k tiles (5-8) cost the weight-gradient
        # blocks occupancy in the step (this standalone timing cannot see it): not candidates
        dgrad = a.b_mode in (L.OPB_ROWN, L.OPB_CONV_DGRAD) and not wgrad
        cands = (1, 2, 3, 4, 5, 7, 9, 10) if wgrad else ((1, 2, 3, 4, 5, 9, 10) if dgrad else
                                                      (1, 2, 3, 4, 5, 6, 7, 8, 9, 10))
        if wgrad and args.wg:  # the weight-gradient kernels with their own split sweep: WG3 (3x3), WGL (linear)
            cands += (32,) if a.b_mode == L.OPB_IM2COL else ((36,) if a.b_mode == L.OPB_ROWN else ())
        if a.a_mode == L.OPA_IM2COL and a.b_mode in (L.OPB_ROWK, L.OPB_CONV_DGRAD):
            # halo tiles (window staged once; split-K by source-channel slices); paired input gradients:
            # 16, 17, 18, 22
            halo = (16, 17, 18, 22) if dgrad else tuple(ops.HALO_TILES)
            cands += tuple(t for t in halo if ops.halo_fits(t, a.conv.batch, a.conv.h, a.conv.w, a.conv.cin,
                                                            a.conv.resample))
        for tile in cands:
            for split in ((1, 2, 4, 8) if 16 <= tile < 32 else (1, 2, 4, 8, 16, 32, 64, 128, 256)):
                if split > 1 and a.K // split < 64:
                    continue
                if 16 <= tile < 32 and not ops.halo_fits(tile, a.conv.batch, a.conv.h, a.conv.w, a.conv.cin,
                                                         a.conv.resample, split):
                    continue
                if wgrad and split > 1 and split * a.M * (a.N + 1) > ops.WS_HALF // 2:
                    continue
                for fold in ((False, True) if split > 1 and not wgrad else (False,)):
                    tt = timeit(a, tile, split, fold)
                    if tt < best_t:
                        best_t, best_tile, best_split, best_fold = tt, tile, split, fold
        k = cat(a)
        tot_cur[k] += cur
        tot_best[k] += best_t
        flops[k] += 2.0 * a.M * a.N * a.K
        done[key] = (cur, best_tile, best_split, best_t, best_fold)
        if key not in table or table[key][2] > best_t:
            table[key] = [best_tile, best_split, best_t, int(best_fold)]
        rows.append((k, a.M, a.N, a.K, a.split_k, a.tile, cur, f"{best_tile}/{best_split}", best_t))
        print(f"[{len(rows)}/{len(calls)}] {k} {a.M}x{a.N}x{a.K} r{a.conv.resample}: {cur:.1f} -> "
              f"{best_tile}/{best_split} {best_t:.1f} us", flush=True)
    # ---- paired backward launches: a layer's weight and input gradient share ONE grid whose
    # workgroups all get the larger tile's LDS, so the dgrad tile (halo tiles: large LDS) and the
    # wgrad tile (128-deep k: 64 KB) are chosen together, timing the pair as the step runs it
    if args.pairs:
        recs = bench.record_gemms(tr)
        seen_p = set()
        orig_pair = L.lib.encdiff_gemm_pair

        def copy_args(a, tile, split, ws_off, fold=False):
            a2 = L.GemmArgs()
            C.memmove(C.byref(a2), C.byref(a), C.sizeof(L.GemmArgs))
            a2.tile, a2.split_k = tile, split
            slab = split > 1 and a2.c_mode in (L.OUT_BF16, L.OUT_F32, L.OUT_F32_ACCUM)
            a2.workspace = ws.data_ptr() + 4 * ws_off if slab else None
            a2.split_counters = (ops._counters().data_ptr() if slab and fold and a2.a_mode != L.OPA_ROWM else None)
            return a2

        def time_pair(w, d):
            for _ in range(2):
                if orig_pair(C.byref(w), C.byref(d), stream) != 0:
                    return float("inf")
            gs = torch.cuda.Stream()
            gs.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=gs):
                st = C.c_void_p(gs.cuda_stream)
                for _ in range(args.reps):
                    orig_pair(C.byref(w), C.byref(d), st)
            g.replay()
            torch.cuda.synchronize()
            s, f = ev(), ev()
            s.record()
            g.replay()
            f.record()
            torch.cuda.synchronize()
            return s.elapsed_time(f) / args.reps * 1e3

        for rec in recs:
            if rec[0] != "pair_ex":
                continue
            w, d = rec[1], rec[2]
            wk, dk = key_of(w), key_of(d)
            if (wk, dk) in seen_p or wk not in table or dk not in table or not selected(d):
                continue
            seen_p.add((wk, dk))
            w_split = table[wk][1]
            conv = d.a_mode == L.OPA_IM2COL
            dc = {(table[dk][0], table[dk][1])} | {(t, s) for t in (1, 2, 3, 4, 5, 9, 10) for s in (1, 2, 4, 8)
                                                   if d.K // s >= 64}
            if conv:
                dc |= {(t, sp) for t in (16, 17, 18, 22) for sp in (1, 2, 4, 8)
                       if ops.halo_fits(t, d.conv.batch, d.conv.h, d.conv.w, d.conv.cin, d.conv.resample, sp)}
            best = None
            for wt in sorted({4, 5, 7, 9, 10, table[wk][0]}):  # tiles 1-3: unpaired (back to back)
                wa = copy_args(w, wt, w_split, 0)
                for dt, ds_ in sorted(dc):
                    if ds_ > 1 and ds_ * d.M * (d.N + 1) + ops.ws_floats(wa) > ops.WS_FLOATS:
                        continue
                    for fold in ((False, True) if ds_ > 1 else (False,)):
                        tt = time_pair(wa, copy_args(d, dt, ds_, ops.ws_floats(wa), fold))
                        if best is None or tt < best[0]:
                            best = (tt, wt, dt, ds_, fold)
            dfold = len(table[dk]) > 3 and bool(table[dk][3])
            cur = time_pair(copy_args(w, table[wk][0], w_split, 0),
                            copy_args(d, table[dk][0], table[dk][1], ops.ws_floats(copy_args(w, table[wk][0], w_split, 0)),
                                      dfold))
            print(f"pair {wk} | {dk}: table {table[wk][0]}/{table[dk][0]}x{table[dk][1]} {cur:.1f} us -> "
                  f"{best[1]}/{best[2]}x{best[3]} {best[0]:.1f} us", flush=True)
            if best[0] < cur:
                table[wk] = [best[1], w_split, table[wk][2]]
                table[dk] = [best[2], best[3], table[dk][2], int(best[4])]
    for cat_name in sorted(tot_cur):
        sel = sorted([r for r in rows if r[0] == cat_name], key=lambda r: -r[6])[:8]
        for r in sel:
            k, M, N, K, s, tile, cur, bt, bb = r
            print(f"{k:10s} M={M:6d} N={N:5d} K={K:6d} split={s:3d} tile={tile} {cur:8.1f}us -> {bt} {bb:8.1f}us "
                  f"({2 * M * N * K / bb / 1e6:7.1f} TF/s)")
    print("category     current_us   best_us   TFLOP/s(best)")
    for k in tot_cur:
        print(f"{k:12s} {tot_cur[k]:9.1f} {tot_best[k]:9.1f} {flops[k] / tot_best[k] / 1e6:8.1f}")
    print(f"TOTAL        {sum(tot_cur.values()):9.1f} {sum(tot_best.values()):9.1f}")
    if args.write_table:
        os.makedirs(os.path.dirname(os.path.abspath(args.write_table)), exist_ok=True)
        json.dump(table, open(args.write_table, "w"), indent=0, sort_keys=True)
        print("wrote", args.write_table)


if __name__ == "__main__":
    main()
