#!/usr/bin/env python3
"""Reduce a rocprofv3 counter_collection.csv (SQ_INSTS_FLAT, SQ_ACTIVE_INST_FLAT, SQ_WAVE_CYCLES,
SQ_INSTS) to one JSON line per kernel: the share of wave cycles spent in FLAT instructions (an upper
bound for scratch spills: global accesses are FLAT too) and FLAT instructions per 1,000.

    python tools/pmc_spill.py OUT/**/counter_collection.csv [--kernel-stats OUT/**/kernel_stats.csv]
"""
import argparse
import collections
import csv
import json


def short(name):
    return name.replace("efl::pl::(anonymous namespace)::", "").replace("efl::(anonymous namespace)::", "") \
        .replace("efl::pl::", "")[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--kernel-stats")
    a = ap.parse_args()
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    with open(a.csv) as f:
        for row in csv.DictReader(f):
            k = row["Kernel_Name"]
            tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
            disp[k].add(row["Dispatch_Id"])
    dur = {}
    if a.kernel_stats:
        with open(a.kernel_stats) as f:
            for row in csv.DictReader(f):
                dur[row["Name"]] = float(row["AverageNs"]) / 1e3
    for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        wave = c.get("SQ_WAVE_CYCLES", 0.0)
        insts = c.get("SQ_INSTS", 0.0)
        print(json.dumps({"kernel": short(k), "dispatches": len(disp[k]),
                          "flat_cycle_share": round(c.get("SQ_ACTIVE_INST_FLAT", 0.0) / wave, 5) if wave else None,
                          "flat_per_1000_insts": round(1000 * c.get("SQ_INSTS_FLAT", 0.0) / insts, 3) if insts else None,
                          "avg_us": round(dur[k], 1) if k in dur else None}))


if __name__ == "__main__":
    main()
