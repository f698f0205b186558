"""The grouped weight-gradient launch of one EncDiff training step: its problems and its time.

    python tools/wgg_probe.py [--batch 128] [--reps 20]

Runs one eager step (B=128 Shapes3D), reads back the planned group(s) of the UNet executor
(encdiff_wgrad_group_plan blobs), prints every problem (body, M, N, K, workgroups, GFLOP) and
times each group launch alone (HIP graph of `reps` launches between events): TFLOP/s and the
fraction of the 2.5 PFLOP/s dense bf16 peak.  ENCDIFF_WGG_ORDER picks the work-item order.
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

KINDS = {0: "WG3 16", 1: "WG3 16 up", 2: "WG3 8", 3: "WG3 8 up", 4: "WG3 4", 5: "WG3 4 up", 6: "WGL",
         7: "gen lin", 8: "gen conv"}
PROB_BYTES = 576  # sizeof(WgProb) in gemm.hip


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--list", action="store_true")
    args = ap.parse_args()
    import encdiff_amd  # noqa: F401
    from encdiff_amd import _lib as L
    from encdiff_amd.configs import model_config
    from encdiff_amd.ldm.util import instantiate_from_config
    from encdiff_amd.trainer import HipTrainer

    torch.manual_seed(0)
    ldm = instantiate_from_config(model_config("shapes3d")).cuda()
    tr = HipTrainer(ldm, args.batch, graph=False)
    tr.init_scale_factor()
    tr.step_eager()
    torch.cuda.synchronize()
    ex = tr.unet._ex
    ev = lambda: torch.cuda.Event(enable_timing=True)
    plans = list(ex._wgg._plans.values())
    detail = len(plans) <= 2
    tot_us = tot_gf = 0.0
    for gi, (host, dev, uprobs) in enumerate(plans):
        raw = bytes(host)
        magic, n_probs, n_items, lds = C.c_int * 4, 0, 0, 0
        hdr = (C.c_int * 4).from_buffer_copy(raw[:16])
        n_probs, n_items = hdr[1], hdr[2]
        probs_off = C.c_long.from_buffer_copy(raw[16:24]).value
        tot_f, tot_b, rows = 0.0, 0, []
        for i in range(n_probs):
            blk = raw[probs_off + i * PROB_BYTES: probs_off + (i + 1) * PROB_BYTES]
            a = uprobs[i]
            kind, gx, nblk = (C.c_int * 3).from_buffer_copy(blk[560:572])
            f = 2.0 * a.M * a.N * a.K
            tot_f += f
            tot_b += nblk
            rows.append((KINDS.get(kind, kind), a.M, a.N, a.K, nblk, f / 1e9, a.conv.h))
        if args.list:
            for r in sorted(rows, key=lambda r: -r[5]):
                print("  %-10s M=%5d N=%5d K=%6d h=%2d blocks=%5d  %.3f GFLOP" % (r[0], r[1], r[2], r[3], r[6], r[4], r[5]))
        by = {}
        for r in rows:
            k = by.setdefault(r[0], [0, 0, 0.0])
            k[0] += 1; k[1] += r[4]; k[2] += r[5]
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())

        def time_blob(hb, db):
            with torch.cuda.stream(st):
                s = C.c_void_p(st.cuda_stream)
                launch = lambda: L.check(L.lib.encdiff_wgrad_group_launch(C.addressof(hb), db.data_ptr(), s), "grp")
                launch()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=st):
                    for _ in range(args.reps):
                        launch()
                g.replay()
                st.synchronize()
                t0, t1 = ev(), ev()
                t0.record(st)
                g.replay()
                t1.record(st)
                st.synchronize()
            return t0.elapsed_time(t1) * 1e3 / args.reps

        def sub_blob(idx):
            arr = (L.GemmArgs * len(idx))(*[probs[i] for i in idx])
            from encdiff_amd import ops
            sc = (ops._workspace().data_ptr() + 4 * ops.WS_HALF, ops.WS_HALF, ops._counters().data_ptr(), ops.COUNTERS)
            nb = C.c_long(0)
            L.check(L.lib.encdiff_wgrad_group_plan(arr, len(idx), *sc, None, 0, C.byref(nb)), "plan")
            hb = (C.c_longlong * ((nb.value + 7) // 8))()
            L.check(L.lib.encdiff_wgrad_group_plan(arr, len(idx), *sc, C.addressof(hb), C.sizeof(hb), C.byref(nb)), "plan")
            return hb, torch.frombuffer(bytearray(hb), dtype=torch.uint8).cuda()

        probs = uprobs  # the callers' problems (the blob holds the planned, slab-redirected ones)
        us = time_blob(host, dev)
        tot_us += us
        tot_gf += tot_f / 1e9
        print(f"group {gi}: {n_probs} problems, {tot_b} workgroups ({n_items} items), {tot_f / 1e9:.1f} GFLOP, "
              f"{us:.1f} us = {tot_f / us / 1e6:.0f} TFLOP/s = {tot_f / us / 1e6 / 2500:.3f} of peak  "
              f"[order {os.environ.get('ENCDIFF_WGG_ORDER', '1')}]")
        if not detail:
            continue
        for k, v in sorted(by.items(), key=lambda kv: -kv[1][2]):
            idx = [i for i, r in enumerate(rows) if r[0] == k]
            t = time_blob(*sub_blob(idx))
            print(f"    {k:10s} {v[0]:3d} problems {v[1]:5d} workgroups {v[2]:7.1f} GFLOP  alone {t:7.1f} us "
                  f"{v[2] * 1e3 / t:6.0f} TFLOP/s")
        # the largest single problems alone
        for i in sorted(range(n_probs), key=lambda i: -rows[i][5])[:8]:
            t = time_blob(*sub_blob([i]))
            r = rows[i]
            print(f"    single {r[0]:10s} M={r[1]} N={r[2]} K={r[3]} blocks={r[4]}: {t:.1f} us "
                  f"{r[5] * 1e3 / t:.0f} TFLOP/s")

    print(f"all groups: {len(plans)} launches, {tot_gf:.1f} GFLOP, {tot_us:.1f} us = {tot_gf * 1e3 / tot_us:.0f} TFLOP/s")


if __name__ == "__main__":
    main()
