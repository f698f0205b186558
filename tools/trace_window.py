"""Summarise a rocprofv3 kernel trace over bench.py's timed region.

    python tools/trace_window.py <run_kernel_trace.csv> --steps K [--top 40]

bench.py launches torch's spin_kernel (torch.cuda._sleep) right before and right after
its timed steps; the region is the span between the last two such marker kernels.  Prints per-kernel calls / total / per-step time.
"""
from __future__ import annotations

import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if "spin_kernel" in r[2]]
    assert len(marks) >= 2, "no marker kernels in trace"
    win = rows[marks[-2] + 1:marks[-1]]
    span = (max(r[1] for r in win) - win[0][0]) / 1e6
    tot = defaultdict(lambda: [0, 0])
    for s, e, n in win:
        tot[n][0] += 1
        tot[n][1] += e - s
    busy = sum(v[1] for v in tot.values()) / 1e6
    lines = [f"window: {len(win)} kernels, span {span:.3f} ms, busy {busy:.3f} ms, steps {a.steps}: "
             f"{span / a.steps:.3f} ms/step span, {busy / a.steps:.3f} ms/step busy",
             f"{'ms/step':>8} {'calls/step':>10} {'avg_us':>8}  kernel"]
    for n, (c, t) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:a.top]:
        lines.append(f"{t / 1e6 / a.steps:8.3f} {c / a.steps:10.1f} {t / c / 1e3:8.1f}  {n[:150]}")
    print("\n".join(lines))
    if a.out:
        open(a.out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
