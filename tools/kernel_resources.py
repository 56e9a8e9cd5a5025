"""Per-kernel register / scratch / LDS use of the gfx950 code objects in libefl_hip.so.

Reads the AMDGPU metadata note (llvm-readelf --notes) of every code object in the library's
.hip_fatbin section and prints one JSON line per kernel: VGPRs (arch + AGPR), SGPRs, spills,
private (scratch) bytes per lane and static LDS. A kernel with spills or scratch is the first
thing to look at when an edit makes it slower.

    python tools/kernel_resources.py [--lib path] [--filter substring]
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_isa_guard import LIB, code_objects  # noqa: E402

READELF = "/opt/rocm/llvm/bin/llvm-readelf"
FIELDS = {
    ".vgpr_count": "vgpr",
    ".agpr_count": "agpr",
    ".sgpr_count": "sgpr",
    ".vgpr_spill_count": "vgpr_spill",
    ".sgpr_spill_count": "sgpr_spill",
    ".private_segment_fixed_size": "scratch_B",
    ".group_segment_fixed_size": "lds_B",
    ".max_flat_workgroup_size": "max_block",
}


def kernels(blob):
    """The amdhsa.kernels list of one code object's metadata note (YAML)."""
    with tempfile.NamedTemporaryFile(suffix=".o") as f:
        f.write(blob)
        f.flush()
        text = subprocess.check_output([READELF, "--notes", f.name]).decode()
    doc = text[text.index("---"):]
    doc = doc[:doc.index("\n...")] if "\n..." in doc else doc
    meta = yaml.safe_load(doc)
    names = [k[".name"] for k in meta["amdhsa.kernels"]]
    plain = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
    for k, name in zip(meta["amdhsa.kernels"], plain):
        row = {"kernel": name}
        row.update({v: k.get(f) for f, v in FIELDS.items()})
        yield row


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=LIB)
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    for blob in code_objects(a.lib):
        for k in kernels(blob):
            if a.filter in k["kernel"]:
                print(json.dumps(k))


if __name__ == "__main__":
    main()
