"""Per-kernel statistics from a rocprofv3 SQLite result (`--kernel-trace` writes `*_results.db`
on this ROCm; `--stats` CSVs only with `--output-format csv`).

    python tools/rocpd_stats.py gpurun_out/x/x_results.db [--per N] [--top 40] [--last K]

--per N divides call counts and times by N (e.g. steps of the traced loop); --last K keeps only
the last K dispatches (a steady-state window after warm-up / capture)."""
from __future__ import annotations

import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--per", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--last", type=int, default=0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    if a.last:
        rows = rows[-a.last:]
    agg = defaultdict(lambda: [0, 0.0])
    for name, s, e in rows:
        agg[name][0] += 1
        agg[name][1] += (e - s) / 1e3
    busy = sum(v[1] for v in agg.values())
    span = (rows[-1][2] - rows[0][1]) / 1e3 if rows else 0.0
    n = sum(v[0] for v in agg.values())
    print(f"window: {n} kernels, span {span / 1e3:.3f} ms, busy {busy / 1e3:.3f} ms; per {a.per:g}: "
          f"{n / a.per:.1f} kernels, busy {busy / a.per / 1e3:.4f} ms, span {span / a.per / 1e3:.4f} ms")
    print(f"{'ms/per':>8} {'calls/per':>10} {'avg_us':>8}  kernel")
    for name, (k, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t / a.per / 1e3:8.4f} {k / a.per:10.1f} {t / k:8.2f}  {name[:150]}")


if __name__ == "__main__":
    main()
