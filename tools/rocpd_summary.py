#!/usr/bin/env python3
"""Per-kernel time summary of a rocprofv3 rocpd database (--kernel-trace output).

    rocpd_summary.py <results.db> [--div N] [--top K] [--since-ms T]

Totals per kernel name (ms, calls, mean us); ``--div`` divides totals (e.g. by the number of
profiled steps); ``--window a:b`` keeps dispatches that start in [a, b) ms after the first one."""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--div", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--window", default=None)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    if not rows:
        print("no kernels")
        return
    t0 = rows[0][1]
    if a.window:
        lo, hi = (float(x) * 1e6 for x in a.window.split(":"))
        rows = [r for r in rows if lo <= r[1] - t0 < hi]
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for name, s, e in rows:
        tot[name] += (e - s) / 1e6
        cnt[name] += 1
    total = sum(tot.values())
    span = (rows[-1][2] - rows[0][1]) / 1e6
    print(f"kernel time {total / a.div:.2f} ms (span {span / a.div:.2f} ms) over {len(rows)} dispatches, /{a.div:g}")
    for name, t in sorted(tot.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f"{t / a.div:9.3f} ms {cnt[name] / a.div:8.1f} calls {1e3 * t / cnt[name]:9.1f} us  {name[:150]}")


if __name__ == "__main__":
    main()
