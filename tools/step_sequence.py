"""Ordered kernel sequence of ONE step from a rocprofv3 kernel trace of bench.py (graph replay).

    python tools/step_sequence.py <run_kernel_trace.csv> --steps K [--out file]

The timed region lies between the last two torch spin_kernel markers (bench.py); the middle
step of it is printed kernel by kernel: start offset, duration, idle gap before it (graph node
launch overhead), plus totals -- busy time, idle time, kernels per step -- and per-name sums.
"""
from __future__ import annotations

import argparse
import csv
import re
from collections import defaultdict


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"\(EncdiffGemmArgs.*", "", n)
    n = re.sub(r"\(Encdiff\w+Args.*", "", n)
    return n[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if "spin_kernel" in r[2]]
    win = rows[marks[-2] + 1:marks[-1]]
    n = len(win) // a.steps
    step = win[n * (a.steps // 2):n * (a.steps // 2 + 1)]
    t0 = step[0][0]
    out = [f"kernels per step {n}; step span {(step[-1][1] - t0) / 1e3:.1f} us"]
    busy = idle = 0
    prev_end = t0
    per = defaultdict(lambda: [0, 0.0, 0.0])
    for s, e, name in step:
        gap = max(0, s - prev_end)
        busy += e - s
        idle += gap
        k = short(name)
        per[k][0] += 1
        per[k][1] += (e - s) / 1e3
        per[k][2] += gap / 1e3
        out.append(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} gap {gap / 1e3:5.1f}  {k}")
        prev_end = max(prev_end, e)
    out.insert(1, f"busy {busy / 1e3:.1f} us, idle gaps {idle / 1e3:.1f} us")
    out.append("\nper kernel: calls, busy us, gap us before")
    for k, (c, b, g) in sorted(per.items(), key=lambda kv: -(kv[1][1] + kv[1][2])):
        out.append(f"{c:5d} {b:9.1f} {g:8.1f}  {k}")
    txt = "\n".join(out)
    if a.out:
        open(a.out, "w").write(txt + "\n")
    print("\n".join(out[:3]))


if __name__ == "__main__":
    main()
