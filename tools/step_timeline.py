#!/usr/bin/env python3
"""GPU timeline of training steps from a rocprofv3 kernel trace: per step (delimited by the AdamW
kernel), the wall time, the union of kernel-busy time (any stream), the idle gaps and the time each
queue is busy, plus the largest idle gaps with the kernels around them.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o run -- python3 bench.py --steps 3 --warmup 2
    python tools/step_timeline.py gpurun_out/tl/.../run_kernel_trace.csv [--gaps 15]
"""
import argparse
import collections
import csv
import glob
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gaps", type=int, default=15)
    ap.add_argument("--marker", default="adamw_kernel")
    a = ap.parse_args()
    path = a.trace if a.trace.endswith(".csv") else glob.glob(a.trace + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         r.get("Queue_Id") or r.get("Stream_Id") or "?"))
    rows.sort()
    ends = [e for s, e, n, q in rows if a.marker in n]
    if len(ends) < 2:
        sys.exit("fewer than two step markers")
    for i in range(1, len(ends)):
        t0, t1 = ends[i - 1], ends[i]
        ks = [r for r in rows if r[0] >= t0 and r[1] <= t1]
        busy, cur_s, cur_e = 0, None, None
        gaps = []
        prev = None
        for s, e, n, q in ks:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                    gaps.append((s - cur_e, prev, n))
                elif s > t0:
                    gaps.append((s - t0, "<step start>", n))
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
            prev = n
        if cur_e is not None:
            busy += cur_e - cur_s
        per_q = collections.Counter()
        for s, e, n, q in ks:
            per_q[q] += e - s
        wall = t1 - t0
        print(f"step {i}: wall {wall / 1e6:.2f} ms, busy (union) {busy / 1e6:.2f} ms, idle {(wall - busy) / 1e6:.2f} ms "
              f"in {len(gaps)} gaps, kernels {len(ks)}; per queue busy: "
              + ", ".join(f"{q}: {v / 1e6:.1f} ms" for q, v in per_q.most_common()))
        if i == len(ends) - 1:
            gaps.sort(reverse=True)
            hist = collections.Counter()
            for g, _, _ in gaps:
                hist["<5us" if g < 5e3 else "5-20us" if g < 2e4 else "20-100us" if g < 1e5 else ">100us"] += g
            print("  idle by gap size:", {k: round(v / 1e6, 2) for k, v in hist.items()}, "ms")
            for g, p, n in gaps[: a.gaps]:
                print(f"  gap {g / 1e3:8.1f} us  after {p[:70]}  before {n[:70]}")


if __name__ == "__main__":
    main()
