#!/usr/bin/env python3
"""HBM bytes per launch of the secret-sharing mask kernels (csrc/mask.hip) from two rocprofv3 PMC
passes (FETCH_SIZE, WRITE_SIZE; separate runs) of `tools/bench_mask.py --no-cpu-baseline`, with the
corrections of tools/pmc_traffic.py (KiB -> bytes, FETCH_SIZE x2 on gfx950 wide streams), next to
the algorithmic bytes. Writes profiles/r01/mask_pmc_traffic.json.

usage: pmc_mask.py <fetch_counter_collection.csv> <write_counter_collection.csv> <elements>
"""
import csv
import json
import os
import sys
from collections import defaultdict

KERNELS = {"k_noise<0>": ("noise", 8), "k_noise<1>": ("share", 12), "k_noise<2>": ("weight_noise", 12),
           "k_mask_cols4": ("mask_cols", 16), "k_mask_rows<4>": ("mask_rows", 16)}


def per_kernel(path, counter):
    vals = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            for key, (name, _) in KERNELS.items():
                if key in row.get("Kernel_Name", ""):
                    vals[name].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    n = int(sys.argv[3])
    out = {"elements": n, "correction": "FETCH_SIZE x2 (gfx950 wide-stream undercount), KiB -> bytes",
           "kernels": {}}
    for name, bpe in KERNELS.values():
        if name in fetch and name in write:
            rd, wr = fetch[name] * 2048, write[name] * 1024
            out["kernels"][name] = {"fetch_bytes": rd, "write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
                                    "algorithmic_bytes": bpe * n, "ratio": round((rd + wr) / (bpe * n), 4)}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "profiles", "r01", "mask_pmc_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
