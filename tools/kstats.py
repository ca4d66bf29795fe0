#!/usr/bin/env python3
"""Print a rocprofv3 kernel_stats.csv as 'total ms, calls, avg us, name' (optionally / N steps)."""
import csv
import sys


def main():
    path = sys.argv[1]
    div = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"sum of kernel time: {tot / 1e6 / div:.2f} ms" + (f" per step (/{div:g})" if div != 1 else ""))
    for r in rows[:top]:
        print(f"{float(r['TotalDurationNs']) / 1e6 / div:9.3f} ms {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:8.1f} us  "
              f"{r['Name'][:100]}")


if __name__ == "__main__":
    main()
