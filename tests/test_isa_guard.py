"""CPU: a static check of the built library's gfx950 machine code.

The Stage-F encode writes its mantissa/exponent streams with `global_store_dwordx4 ... nt sc1`,
emitted from inline asm (csrc/fxp.hip `st<>`; clang has no builtin for the sc1 bit). The compiler's
hazard recognizer cannot see an asm store, so the asm itself pads it with `s_nop 1`: a VALU write
to the store's data VGPRs right after a >8-byte store needs a wait state on gfx950, and round 1
saw wrong bits when it was missing. This test disassembles every code object in
libefl_hip.so and fails if any such store is not immediately followed by its s_nop — whatever the
register allocation around it does after a future edit.
"""
import os
import re
import struct
import subprocess

import pytest

from conftest import PKG

LIB = os.path.join(PKG, "efl", "libefl_hip.so")
OBJDUMP = "/opt/rocm/llvm/bin/llvm-objdump"
EM_AMDGPU = 224


def code_objects(path):
    """The AMDGPU ELF code objects inside the .so's .hip_fatbin section."""
    out = subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", path, "/dev/stdout"],
                         check=True, capture_output=True).stdout
    objs = []
    i = 0
    while True:
        j = out.find(b"\x7fELF", i)
        if j < 0:
            break
        i = j + 4
        if out[j + 4] != 2:                       # ELFCLASS64
            continue
        (machine,) = struct.unpack_from("<H", out, j + 0x12)
        if machine != EM_AMDGPU:
            continue
        (shoff,) = struct.unpack_from("<Q", out, j + 0x28)
        shentsize, shnum = struct.unpack_from("<HH", out, j + 0x3A)
        objs.append(out[j:j + shoff + shentsize * shnum])
        i = j + shoff + shentsize * shnum
    return objs


@pytest.fixture(scope="module")
def disassembly(tmp_path_factory):
    if not os.path.exists(OBJDUMP):
        pytest.skip("llvm-objdump not in this image")
    d = tmp_path_factory.mktemp("isa")
    texts = []
    for k, blob in enumerate(code_objects(LIB)):
        p = d / f"co{k}.o"
        p.write_bytes(blob)
        texts.append(subprocess.check_output([OBJDUMP, "-d", "--mcpu=gfx950", str(p)]).decode())
    assert texts, "no gfx950 code object found in libefl_hip.so"
    return texts


STORE = re.compile(r"^\s*global_store_dwordx([24])\b.*\bnt sc1\b")
INSN = re.compile(r"^\s+([a-z_][a-z0-9_]*)\b")


def test_every_asm_nt_sc1_store_is_padded(disassembly):
    n_checked = 0
    for text in disassembly:
        insns = [ln for ln in text.splitlines() if INSN.match(ln)]
        for i, ln in enumerate(insns):
            if STORE.match(ln):
                n_checked += 1
                nxt = insns[i + 1] if i + 1 < len(insns) else ""
                m = re.match(r"^\s+s_nop\s+(\d+)", nxt)
                assert m and int(m.group(1)) >= 1, f"unpadded store:\n{ln}\nfollowed by\n{nxt}"
    # the default fp32 encode (streaming + batched) uses the flavour, so the check is not vacuous
    assert n_checked >= 16, n_checked
