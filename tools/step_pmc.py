"""MFMA utilisation of every kernel family in ONE eager training step, from SQ counters.

    # on the GPU box (one --pmc group per run, kernel trace in the same run):
    rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES ... --output-format csv \
        -d gpurun_out/step_pmc -o run -- python3 tools/step_pmc.py --run
    python3 tools/step_pmc.py --report gpurun_out/step_pmc [--out profiles/r06_step_mfma_pmc.txt]

--run builds the bench model (shapes3d, B=128), runs two warm eager steps, then ONE step bracketed
by torch spin_kernel markers.  --report keeps the dispatches between the last two markers and
prints, per kernel name: calls, summed duration, MFMA instructions, SQ_VALU_MFMA_BUSY_CYCLES,
and the MFMA pipe utilisation  u = N_mfma * 16 cyc / (duration * 2.4 GHz * 1024 SIMDs)
(v_mfma_f32_16x16x32_bf16 occupies a SIMD's matrix pipe for 16 cycles: 16384 flop at the
2.5 PFLOP/s dense bf16 peak; the BUSY/N_mfma column checks that reading of the counter).
Durations come from the counter run's kernel trace (dispatches serialised by the profiler).
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CLK_GHZ = 2.4
SIMDS = 1024
MFMA_CYC = 16


def run(batch):
    import torch
    import bench
    from encdiff_amd.trainer import HipTrainer
    ldm, _ = bench.build_ldm("shapes3d")
    tr = HipTrainer(ldm, batch, graph=False, pool_size=480000)
    tr.init_scale_factor()
    for _ in range(2):
        tr.step()
    torch.cuda.synchronize()
    torch.cuda._sleep(1000)
    tr.step()
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    print("step done")


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"\(Encdiff\w+.*", "", n)
    n = re.sub(r"void ", "", n)
    return n[:88]


def family(n):
    for f in ("st_wgrad", "wgrad_group", "wgrad3x3", "wgradlin", "gemm_finalize", "gemm2", "gemm", "resconv",
              "st_tail", "st_head", "attn", "conv", "gn_", "ln_", "bn_", "adamw"):
        if f in n:
            return f
    return "other"


def report(d, out):
    kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    cc = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not kt or not cc:
        sys.exit(f"no kernel_trace / counter_collection csv under {d}")
    disp = {}
    for r in csv.DictReader(open(kt[0])):
        disp[int(r["Dispatch_Id"])] = (r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    marks = sorted(i for i, (n, _) in disp.items() if "spin_kernel" in n)
    if len(marks) < 2:
        sys.exit("step markers not found")
    lo, hi = marks[-2], marks[-1]
    ctr = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(cc[0])):
        i = int(r["Dispatch_Id"])
        if lo < i < hi:
            ctr[i][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = defaultdict(lambda: defaultdict(float))
    for i in range(lo + 1, hi):
        if i not in disp:
            continue
        n, ns = disp[i]
        a = agg[short(n)]
        a["calls"] += 1
        a["ns"] += ns
        for k, v in ctr[i].items():
            a[k] += v
    lines = []
    hdr = f"{'kernel':88s} {'calls':>5s} {'us':>8s} {'N_mfma':>10s} {'busy/N':>6s} {'util':>6s} {'TF/s':>6s} {'valu/mfma':>9s}"
    lines.append(hdr)
    fam = defaultdict(lambda: defaultdict(float))
    for n, a in sorted(agg.items(), key=lambda kv: -kv[1]["ns"]):
        nm = a.get("SQ_INSTS_MFMA", 0.0)
        us = a["ns"] / 1e3
        util = nm * MFMA_CYC / (a["ns"] * CLK_GHZ * SIMDS) if a["ns"] else 0.0
        tf = nm * 16384 / a["ns"] / 1e3 if a["ns"] else 0.0
        bpn = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / nm if nm else 0.0
        vpm = a.get("SQ_INSTS_VALU", 0.0) / nm if nm else 0.0
        lines.append(f"{n:88s} {int(a['calls']):5d} {us:8.1f} {nm:10.0f} {bpn:6.1f} {util:6.3f} {tf:6.1f} {vpm:9.2f}")
        f = fam[family(n)]
        f["ns"] += a["ns"]
        f["mfma"] += nm
        f["calls"] += a["calls"]
    lines.append("")
    lines.append(f"{'family':12s} {'calls':>5s} {'us':>8s} {'util':>6s} {'TF/s':>6s}")
    tot = defaultdict(float)
    for k, f in sorted(fam.items(), key=lambda kv: -kv[1]["ns"]):
        util = f["mfma"] * MFMA_CYC / (f["ns"] * CLK_GHZ * SIMDS)
        lines.append(f"{k:12s} {int(f['calls']):5d} {f['ns'] / 1e3:8.1f} {util:6.3f} {f['mfma'] * 16384 / f['ns'] / 1e3:6.1f}")
        for kk in ("ns", "mfma", "calls"):
            tot[kk] += f[kk]
    lines.append(f"{'step':12s} {int(tot['calls']):5d} {tot['ns'] / 1e3:8.1f} "
                 f"{tot['mfma'] * MFMA_CYC / (tot['ns'] * CLK_GHZ * SIMDS):6.3f} {tot['mfma'] * 16384 / tot['ns'] / 1e3:6.1f}")
    txt = "\n".join(lines)
    print(txt)
    if out:
        with open(out, "w") as fh:
            fh.write(__doc__.split("\n\n")[0] + "\n\n" + txt + "\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--report", default="")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    if a.run:
        run(a.batch)
    if a.report:
        report(a.report, a.out)


if __name__ == "__main__":
    main()
