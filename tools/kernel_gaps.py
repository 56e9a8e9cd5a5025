#!/usr/bin/env python3
"""Per kernel name in a rocprofv3 kernel_trace.csv: dispatches, mean duration and the mean idle gap
between the previous dispatch's end and this one's start (same queue order), in microseconds. Used
to tell kernel time from the time between kernels (tools/config3_probe.py's batched vs streaming
steps). One JSON document."""
import collections
import csv
import json
import sys


def main():
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    agg = collections.defaultdict(lambda: {"n": 0, "dur": 0.0, "gap": 0.0})
    prev_end = None
    for s, e, k in rows:
        name = k.replace("efl::(anonymous namespace)::", "")[:80]
        a = agg[name]
        a["n"] += 1
        a["dur"] += (e - s) / 1e3
        if prev_end is not None:
            a["gap"] += max(0, s - prev_end) / 1e3
        prev_end = e
    out = {k: {"dispatches": v["n"], "avg_us": round(v["dur"] / v["n"], 2), "avg_gap_before_us": round(v["gap"] / v["n"], 2)}
           for k, v in agg.items() if "batched" in k or "k_stream" in k}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
