"""HBM traffic of the GEMM family (bench.py's roofline kernel) from rocprofv3 PMC passes.

Run (GPU box), one counter per pass as MI355X_MICROARCH.md prescribes (FETCH_SIZE and
WRITE_SIZE do not fit one pass):

    cd /tmp && export TMPDIR=/tmp
    rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_f -o run -- python3 $R/tools/gemm_traffic.py run
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_w -o run -- python3 $R/tools/gemm_traffic.py run
    python tools/gemm_traffic.py summarize gpurun_out/pmc_f gpurun_out/pmc_w --out profiles/gemm_traffic.json

(`run --config celeba128` for configs[4]; summarize it into profiles/gemm_traffic_celeba128.json,
which is the file bench.py --config celeba128 reads.)

`run` records the GEMM launches of one eager training step (B=128) and replays them once
between torch spin_kernel markers, preceded by a calibration copy of known size (the
ENCDIFF_EW_COPY kernel, 16-B lanes, 256 MiB read + 256 MiB write).  `summarize` sums the
counters of the gemm dispatches between the markers, converts them with the calibration
copy's bytes-per-unit (the guide: FETCH_SIZE reports 1/2 of a 16-B-lane streaming read on
gfx950), and writes bytes per launch next to the algorithmic bytes per launch.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

CAL_BYTES = 256 << 20


def run(batch: int, config: str = "shapes3d"):
    import torch
    import bench
    from encdiff_amd import ops
    from encdiff_amd.trainer import HipTrainer
    torch.cuda.set_device(0)
    ldm, _ = bench.build_ldm(config)
    tr = HipTrainer(ldm, batch, graph=False)
    tr.init_scale_factor()
    tr.step_eager()
    calls = bench.record_gemms(tr)
    n = CAL_BYTES // 2
    src = torch.randn(n // 64, 64, device="cuda").to(torch.bfloat16)
    dst = torch.empty_like(src)
    torch.cuda.synchronize()
    torch.cuda._sleep(1000)
    ops.ew(0, src, dst)                      # calibration: ENCDIFF_EW_COPY
    for c in calls:                          # a spin marker before every call: per-call segments
        torch.cuda._sleep(1)
        bench.replay_gemms([c])
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    probs = bench.gemm_problems(calls)
    alg = sum(bench.gemm_alg_bytes(a) for a in probs)

    def desc(a):
        return {"M": a.M, "N": a.N, "K": a.K, "a_mode": a.a_mode, "b_mode": a.b_mode, "c_mode": a.c_mode,
                "tile": a.tile, "split_k": a.split_k, "hw": [a.conv.h, a.conv.w], "cin": a.conv.cin,
                "resample": a.conv.resample, "alg_bytes": bench.gemm_alg_bytes(a), "flops": 2.0 * a.M * a.N * a.K}
    per_call = []
    for c in calls:
        ps = [c[1]] if c[0] == "gemm" else ([c[1], c[2]] if c[0] == "pair_ex" else (c[3] if c[0] in ("group", "stwg") else []))
        per_call.append({"kind": c[0], "problems": [desc(a) for a in ps]})
    with open(os.path.join(REPO, "gpurun_out", "gemm_traffic_calls.json"), "w") as f:
        json.dump({"launches": len(calls), "alg_bytes": alg, "batch": batch, "config": config,
                   "flops": sum(2.0 * a.M * a.N * a.K for a in probs), "calls": per_call}, f)
    print(f"replayed {len(calls)} gemm launches")


def _rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    assert files, f"no counter_collection.csv under {d}"
    out = []
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                out.append((int(r["Dispatch_Id"]), r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"])))
    out.sort()
    return out


def _segments(rows, counter):
    """rows between the first and the last spin marker, split at every marker: segment 0 is the
    calibration copy, segment i + 1 the dispatches of recorded call i."""
    marks = [i for i, r in enumerate(rows) if "spin_kernel" in r[1]]
    assert len(marks) >= 3, "markers missing"
    segs = []
    for a, b in zip(marks[:-1], marks[1:]):
        segs.append([r for r in rows[a + 1:b] if r[2] == counter])
    return segs


FAM = ("gemm_kernel", "gemm2_kernel", "gemm_finalize", "wgrad3x3_kernel", "wgradlin_kernel", "wgrad_group_kernel", "st_wgrad_kernel", "st_wgrad_fold")


def _window(rows, counter):
    segs = _segments(rows, counter)
    cal = [r for r in segs[0] if "ew_kernel" in r[1]]
    # single, paired, split-K finalize kernels, and the weight-gradient kernels (WG3 3x3 conv, WGL linear)
    gem = [r for s in segs[1:] for r in s if any(k in r[1] for k in FAM)]
    launches = len({r[0] for r in gem})
    return sum(r[3] for r in cal), sum(r[3] for r in gem), launches, segs


def summarize(fdir, wdir, out):
    f_cal, f_gemm, n1, fseg = _window(_rows(fdir), "FETCH_SIZE")
    w_cal, w_gemm, n2, wseg = _window(_rows(wdir), "WRITE_SIZE")
    assert n1 == n2, (n1, n2)
    rd = f_gemm * CAL_BYTES / f_cal        # calibrated: units of the counter -> bytes
    wr = w_gemm * CAL_BYTES / w_cal
    meta = json.load(open(os.path.join(REPO, "gpurun_out", "gemm_traffic_calls.json")))
    n = meta["launches"]  # API calls (bench.py's launches_per_step); n1 = kernel dispatches
    res = {"launches": n, "dispatches": n1, "read_bytes_per_step": rd, "write_bytes_per_step": wr,
           "bytes_per_launch": (rd + wr) / n, "alg_bytes_per_launch": meta["alg_bytes"] / n,
           "traffic_over_alg": (rd + wr) / meta["alg_bytes"],
           "fetch_units_per_cal_byte": f_cal / CAL_BYTES, "write_units_per_cal_byte": w_cal / CAL_BYTES,
           "batch": meta.get("batch", 128), "config": meta.get("config", "shapes3d"),
           "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes of tools/gemm_traffic.py run "
                     f"({meta.get('config', 'shapes3d')}, B={meta.get('batch', 128)}), "
                     "calibrated on a 256 MiB 16-B-lane copy"}
    # per call: measured read / write bytes beside the algorithmic bytes, and per kernel name
    calls = meta.get("calls", [])
    if len(calls) == len(fseg) - 1 == len(wseg) - 1:
        rows, byk = [], {}
        for i, c in enumerate(calls):
            fr = [r for r in fseg[i + 1] if any(k in r[1] for k in FAM)]
            r_b = sum(r[3] for r in fr) * CAL_BYTES / f_cal
            w_b = sum(r[3] for r in wseg[i + 1] if any(k in r[1] for k in FAM)) * CAL_BYTES / w_cal
            alg = sum(p["alg_bytes"] for p in c["problems"])
            ks = sorted({r[1].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0] for r in fr})
            rows.append({"i": i, "kind": c["kind"], "kernels": ks, "read": r_b, "write": w_b, "alg": alg,
                         "ratio": (r_b + w_b) / alg if alg else None,
                         "problems": [{k: p[k] for k in ("M", "N", "K", "a_mode", "b_mode", "c_mode", "tile",
                                                         "split_k", "hw", "cin")} for p in c["problems"]]})
            for k in ks:
                e = byk.setdefault(k, {"calls": 0, "read": 0.0, "write": 0.0, "alg": 0.0})
                e["calls"] += 1
                e["read"] += r_b / len(ks)
                e["write"] += w_b / len(ks)
                e["alg"] += alg / len(ks)
        res["by_kernel"] = dict(sorted(byk.items(), key=lambda kv: -(kv[1]["read"] + kv[1]["write"])))
        res["worst_calls"] = sorted(rows, key=lambda r: -(r["read"] + r["write"] - r["alg"]))[:25]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k not in ("worst_calls",)}, indent=1))


def _kname(n):
    return n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def pmc(adir, bdir, out, traffic):
    """Per-kernel-class SQ / L2 counters of the replay (two --pmc passes, each with --kernel-trace):
    MFMA pipe utilisation, occupancy, wait shares and L2 hit rate beside the measured HBM traffic.

    util  = SQ_INSTS_MFMA * 16 cyc / (duration * 2.4 GHz * 1024 SIMDs)  (16x16x32 bf16: 16 cycles;
            the busy/N column = SQ_VALU_MFMA_BUSY_CYCLES / SQ_INSTS_MFMA checks that reading)
    occ   = SQ_WAVE_CYCLES * 4 / (duration cycles * 256 CUs): mean resident waves per CU
            (SQ_WAVE_CYCLES counts quad-cycles, MI355X_MICROARCH.md)
    wait  = SQ_WAIT_ANY / SQ_WAVE_CYCLES, issue = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES,
    ldsw  = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES, L2hit = TCC_HIT / (TCC_HIT + TCC_MISS)."""
    agg = {}

    def add(d):
        kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
        assert kt, f"no kernel_trace.csv under {d}"
        names, dur = {}, {}
        for r in csv.DictReader(open(kt[0])):
            names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
            dur[int(r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        marks = sorted(i for i, n in names.items() if "spin_kernel" in n)
        lo, hi = marks[1], marks[-1]            # skip the calibration segment
        rows = _rows(d)
        seen = set()
        for i, n, c, v in rows:
            if not (lo < i < hi) or not any(k in n for k in FAM):
                continue
            e = agg.setdefault(_kname(n), {"calls": {}, "ctr": {}})
            e["ctr"][c] = e["ctr"].get(c, 0.0) + v
            if i not in seen and d == adir:
                seen.add(i)
                e["calls"][i] = dur.get(i, 0)
    add(adir)
    add(bdir)
    byk = {}
    if traffic and os.path.exists(traffic):
        byk = json.load(open(traffic)).get("by_kernel", {})
    lines = [pmc.__doc__.split("\n\n")[0].strip(), "",
             f"{'kernel':52s} {'calls':>5s} {'us':>7s} {'util':>6s} {'busy/N':>6s} {'occ':>5s} {'wait':>5s} "
             f"{'issue':>5s} {'ldsw':>5s} {'L2hit':>5s} {'valu/mfma':>9s} {'traffic/alg':>11s} {'GB/s':>6s}"]
    tot_ns = tot_m = 0.0
    for k, e in sorted(agg.items(), key=lambda kv: -sum(kv[1]["calls"].values())):
        ns = float(sum(e["calls"].values()))
        if not ns:
            continue
        c = e["ctr"]
        nm = c.get("SQ_INSTS_MFMA", 0.0)
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        cyc = ns * 2.4
        hit, miss = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
        t = byk.get(k, {})
        rw = t.get("read", 0.0) + t.get("write", 0.0)
        ratio = f"{rw / t['alg']:11.2f}" if t.get("alg") else f"{'-':>11s}"
        gbs = rw / ns if rw else 0.0
        lines.append(f"{k[:52]:52s} {len(e['calls']):5d} {ns / 1e3:7.1f} {nm * 16 / (cyc * 1024):6.3f} "
                     f"{(c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0.0) / nm if nm else 0.0):6.1f} "
                     f"{wc * 4 / (cyc * 256):5.1f} {c.get('SQ_WAIT_ANY', 0.0) / wc:5.2f} "
                     f"{c.get('SQ_ACTIVE_INST_ANY', 0.0) / wc:5.2f} {c.get('SQ_WAIT_INST_LDS', 0.0) / wc:5.2f} "
                     f"{(hit / (hit + miss) if hit + miss else 0.0):5.2f} "
                     f"{(c.get('SQ_INSTS_VALU', 0.0) / nm if nm else 0.0):9.2f} {ratio} {gbs:6.0f}")
        tot_ns += ns
        tot_m += nm
    lines.append(f"{'GEMM family':52s} {'':5s} {tot_ns / 1e3:7.1f} {tot_m * 16 / (tot_ns * 2.4 * 1024):6.3f}")
    txt = "\n".join(lines) + "\n"
    print(txt)
    with open(out, "w") as f:
        f.write(txt)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["run", "summarize", "pmc"])
    ap.add_argument("dirs", nargs="*")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--config", default="shapes3d", choices=["shapes3d", "celeba128"])
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "gemm_traffic.json"))
    a = ap.parse_args()
    if a.mode == "run":
        os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
        run(a.batch, a.config)
    elif a.mode == "pmc":
        pmc(a.dirs[0], a.dirs[1], a.out, a.dirs[2] if len(a.dirs) > 2 else "")
    else:
        summarize(a.dirs[0], a.dirs[1], a.out)


if __name__ == "__main__":
    main()
