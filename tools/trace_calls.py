"""Split a rocprofv3 kernel trace (run_kernel_trace.csv) into host calls and show where each call's
wall time goes: the kernels it launched (short names, grid, VGPRs, duration) and the gaps between
them. A new call starts wherever the GPU sat idle longer than --gap-us, or at a kernel whose short
name is given with --first.

    python tools/trace_calls.py gpurun_out/r05_crtkt/run_kernel_trace.csv [--match pl::] [--last 3]
"""
import argparse
import csv
import re
import statistics


def short(name):
    name = re.sub(r"\(.*$", "", name.replace("(anonymous namespace)::", ""))
    name = name.replace("void ", "").replace("efl::pl::", "").replace("efl::", "")
    return name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="", help="keep kernels whose full name contains this")
    ap.add_argument("--gap-us", type=float, default=50.0)
    ap.add_argument("--first", default="", help="a kernel (short-name prefix) that opens a call")
    ap.add_argument("--last", type=int, default=3, help="print this many calls in full")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            if a.match and a.match not in r["Kernel_Name"]:
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), int(r["VGPR_Count"]),
                         int(r["Accum_VGPR_Count"])))
    rows.sort()
    calls, cur = [], []
    for r in rows:
        if cur and (r[0] - cur[-1][1] > a.gap_us * 1e3 or (a.first and r[2].startswith(a.first))):
            calls.append(cur)
            cur = []
        cur.append(r)
    if cur:
        calls.append(cur)
    sig = {}
    for c in calls:
        sig.setdefault(tuple(k[2] for k in c), []).append(c)
    for names, cs in sig.items():
        span = [c[-1][1] - c[0][0] for c in cs]
        busy = [sum(k[1] - k[0] for k in c) for c in cs]
        print(f"{len(cs)} calls of {len(names)} kernels: span median {statistics.median(span) / 1e3:.1f} us, "
              f"kernels {statistics.median(busy) / 1e3:.1f} us, gaps {statistics.median(s - b for s, b in zip(span, busy)) / 1e3:.1f} us")
        for j, nm in enumerate(names):
            d = [c[j][1] - c[j][0] for c in cs]
            g = [c[j][0] - c[j - 1][1] for c in cs] if j else [0]
            k = cs[0][j]
            print(f"   {nm:60s} wg {k[3]:7d} vgpr {k[4]:3d}+{k[5]:3d}  {statistics.median(d) / 1e3:9.1f} us"
                  f"  (gap before {statistics.median(g) / 1e3:6.1f} us)")


if __name__ == "__main__":
    main()
