#!/usr/bin/env python3
"""Turn two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs, csv) of
`bench.py --no-cpu-baseline` into profiles/pmc_traffic.json: HBM bytes per launch of each Stage-F
kernel. Per MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE
reports exactly half of a wide coalesced streaming read, so it is doubled; WRITE_SIZE reads exactly
for 16-B-per-lane stores.

usage: pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> <elements> [profile_dir]

The JSON records where it came from (profile_dir, the library's build hash, the command), which
bench.py copies into its line as roofline.traffic_source.
"""
import csv
import json
import os
import sys
from collections import defaultdict


def per_kernel(path, counter):
    vals = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            name = row.get("Kernel_Name", "")
            kind = "encode" if "Enc" in name else "decode" if "Dec" in name else None
            if kind and "k_stream" in name:
                vals[kind].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items() if v}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    n = int(sys.argv[3])
    prof_dir = sys.argv[4] if len(sys.argv) > 4 else ""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "elastic-federated-learning-solution_amd"))
    try:
        from efl import lib as efl_lib
        library = efl_lib.version()
    except Exception:   # no library here: leave the field empty
        library = None
    out = {"elements": n, "source": [os.path.basename(sys.argv[1]), os.path.basename(sys.argv[2])],
           "profile_dir": prof_dir, "library": library,
           "command": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) -- "
                      "python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras",
           "correction": "FETCH_SIZE x2 (gfx950 wide-stream undercount), KiB -> bytes", "kernels": {}}
    for k in ("encode", "decode"):
        if k in fetch and k in write:
            rd = fetch[k] * 1024 * 2
            wr = write[k] * 1024
            out["kernels"][k] = {"fetch_bytes": rd, "write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
                                 "algorithmic_bytes": 20 * n}
    with open(os.path.join(root, "profiles", "pmc_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
