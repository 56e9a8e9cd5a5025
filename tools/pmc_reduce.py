#!/usr/bin/env python3
"""Reduce a rocprofv3 output directory to a small JSON summary and (with --prune) delete the bulky
CSVs: per kernel, the dispatch count, every counter summed over dispatches and divided by them
(counter_collection.csv), and the kernel-trace statistics (kernel_stats.csv). Keeps gpurun_out/
under the size the harness copies back.

    python tools/pmc_reduce.py DIR [--match SUBSTR ...] [--prune] > summary.json
"""
import argparse
import collections
import csv
import glob
import json
import os
import shutil


def short(name):
    for p in ("efl::pl::(anonymous namespace)::", "efl::(anonymous namespace)::", "efl::pl::"):
        name = name.replace(p, "")
    return name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", nargs="*", default=[])
    ap.add_argument("--prune", action="store_true")
    a = ap.parse_args()
    out = {"dir": a.dir, "kernels": {}}
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        tot = collections.defaultdict(lambda: collections.defaultdict(float))
        disp = collections.defaultdict(set)
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                if a.match and not any(m in k for m in a.match):
                    continue
                tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[k].add(row["Dispatch_Id"])
        for k, c in tot.items():
            n = len(disp[k])
            e = out["kernels"].setdefault(k, {})
            e["dispatches"] = n
            e.setdefault("per_dispatch", {}).update({cn: v / n for cn, v in c.items()})
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_stats.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Name"])
                if a.match and not any(m in k for m in a.match):
                    continue
                out["kernels"].setdefault(k, {})["stats"] = {
                    "calls": int(row["Calls"]), "avg_us": float(row["AverageNs"]) / 1e3,
                    "min_us": float(row["MinNs"]) / 1e3, "max_us": float(row["MaxNs"]) / 1e3}
    print(json.dumps(out, indent=1))
    if a.prune:
        shutil.rmtree(a.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
