"""Ordered kernel sequence of ONE DDIM sampler step from a rocprofv3 kernel trace (csv) of
tools/ddim_prof.py: the kernels between the last two ddim_kernel launches.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/ddim_prof.py --steps 20
    python tools/ddim_sequence.py OUT/.../run_kernel_trace.csv [--out file]
"""
from __future__ import annotations

import argparse
import csv
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from step_sequence import short  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if "ddim_kernel" in r[2]]
    step = rows[marks[-2] + 1:marks[-1] + 1]
    t0 = step[0][0]
    out = [f"kernels per DDIM step {len(step)}; span {(step[-1][1] - t0) / 1e3:.1f} us"]
    sums = defaultdict(lambda: [0, 0.0])
    prev = t0
    for s, e, n in step:
        out.append(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} gap {(s - prev) / 1e3:5.1f}  {short(n)}")
        sums[short(n)][0] += 1
        sums[short(n)][1] += (e - s) / 1e3
        prev = e
    out.append("per kernel: calls, busy us")
    for k, (c, t) in sorted(sums.items(), key=lambda kv: -kv[1][1]):
        out.append(f"{c:5d} {t:8.1f}  {k}")
    txt = "\n".join(out)
    if a.out:
        open(a.out, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
