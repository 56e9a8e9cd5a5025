"""Inner loops of one kernel in libefl_hip.so's gfx950 code: every backward branch, its body's
instruction count and mix (VALU products vs moves vs scratch / LDS / memory traffic).

    python tools/isa_loops.py k_matmul28ILi32ELi2E [--top 12]

The argument is a substring of the mangled kernel name. Used to check that a hot loop holds no
scratch spills and how many non-product VALU instructions ride along each limb product.
"""
import argparse
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_isa_guard import LIB, OBJDUMP, backward_loops, code_objects, kernel_instructions, loop_mix  # noqa: E402,E501

def kernel_lines(name, lib=LIB):
    texts = []
    for blob in code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".o") as f:
            f.write(blob)
            f.flush()
            texts.append(subprocess.check_output([OBJDUMP, "-d", "--mcpu=gfx950", f.name]).decode())
    ins = kernel_instructions(texts, name)
    if ins is None:
        raise SystemExit("kernel not found: " + name)
    return ins


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--lib", default=LIB, help="library to disassemble (default: the built libefl_hip.so)")
    a = ap.parse_args()
    ins = kernel_lines(a.kernel, a.lib)
    for t, k in backward_loops(ins):
        mix = loop_mix(ins, (t, k))
        print(f"loop [{t}, {k}] {k + 1 - t} insns:", ", ".join(f"{o} {n}" for o, n in mix.most_common(a.top)))

if __name__ == "__main__":
    main()
