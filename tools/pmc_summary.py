#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs: per kernel (name prefix), per counter, the mean over
dispatches of the per-dispatch value (summed over the dispatch's rows), plus derived clock.
Usage: pmc_summary.py <dir-with-*/run_counter_collection.csv> [kernel-substring]"""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
for f in sorted(glob.glob(f"{root}/*/run_counter_collection.csv")):
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
    dur = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if sub and sub not in k:
            continue
        key = (k[:60], r["Dispatch_Id"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        if "End_Timestamp" in r and r.get("Start_Timestamp"):
            dur[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    agg = defaultdict(lambda: defaultdict(list))
    for (k, d), cs in per.items():
        for c, v in cs.items():
            agg[k][c].append(v)
        if (k, d) in dur:
            agg[k]["_ns"].append(dur[(k, d)])
    for k, cs in agg.items():
        vals = {c: sum(v) / len(v) for c, v in cs.items()}
        extra = ""
        if "GRBM_GUI_ACTIVE" in vals and vals.get("_ns"):
            extra = f" clock={vals['GRBM_GUI_ACTIVE'] / 8 / vals['_ns'] * 1e3:.0f}MHz"
        print(f.split('/')[-2], k, " ".join(f"{c}={v:.4g}" for c, v in sorted(vals.items())), extra)
