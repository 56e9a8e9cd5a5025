"""CPU: a static check of the built library's gfx950 machine code.

The Stage-F encode writes its mantissa/exponent streams with `global_store_dwordx4 ... nt sc1`,
emitted from inline asm (csrc/fxp.hip `st<>`; clang has no builtin for the sc1 bit). The compiler's
hazard recognizer cannot see an asm store, so the asm itself pads it with `s_nop 1`: a VALU write
to the store's data VGPRs right after a >8-byte store needs a wait state on gfx950, and round 1
saw wrong bits when it was missing. This test disassembles every code object in
libefl_hip.so and fails if any such store is not immediately followed by its s_nop — whatever the
register allocation around it does after a future edit.

The Paillier kernels run at a 256-VGPR cap (two waves per SIMD) and some spill; the second test
checks that the spills stay out of the radix-2^28 Montgomery row (the loop that issues the
v_mad_u64_u32 products) of the default-family hot kernels, and that the row stays mostly products.
"""
import collections
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


LINE = re.compile(r"^\s+([a-z_][a-z0-9_]*)\b(.*?)//\s*([0-9A-Fa-f]+):")
BRANCH = re.compile(r"^(s_cbranch_\w+|s_branch)$")


def kernel_instructions(texts, name):
    """(address, opcode, operands) of the first kernel whose symbol contains `name`."""
    for text in texts:
        lines = text.split("\n")
        for i, ln in enumerate(lines):
            if re.match(r"^[0-9a-f]+ <.*%s.*>:" % re.escape(name), ln):
                out = []
                for m in lines[i + 1:]:
                    if re.match(r"^[0-9a-f]+ <", m):
                        break
                    g = LINE.match(m)
                    if g:
                        out.append((int(g.group(3), 16), g.group(1), g.group(2).strip()))
                return out
    return None


def backward_loops(ins):
    """[(first, last)] instruction index ranges closed by a backward branch."""
    index = {addr: k for k, (addr, _, _) in enumerate(ins)}
    loops = []
    for k, (addr, op, args) in enumerate(ins):
        if not BRANCH.match(op):
            continue
        imm = int(args.split()[0])
        imm = imm - 0x10000 if imm >= 0x8000 else imm
        t = index.get(addr + 4 + 4 * imm)
        if imm < 0 and t is not None:
            loops.append((t, k))
    return loops


def loop_mix(ins, loop):
    return collections.Counter(op for _, op, _ in ins[loop[0]:loop[1] + 1])


# default-family (C = 32) kernels of the n^2 ops at 1024 / 4096-bit n and of decryption
HOT = ["k_encrypt28ILi32ELi2E", "k_encrypt28ILi32ELi8E", "k_fbpowm28ILi32ELi2E", "k_tomont28ILi32ELi2E",
       "k_matmul28ILi32ELi2E", "k_decryptILi32ELi1E", "k_decryptILi32ELi4E"]


@pytest.mark.parametrize("kernel", HOT)
def test_montgomery_row_has_no_spills(disassembly, kernel):
    ins = kernel_instructions(disassembly, "pl12_GLOBAL__N_1" + str(len(kernel.split("ILi")[0])) + kernel)
    assert ins, kernel
    rows = []
    for lp in backward_loops(ins):
        mix = loop_mix(ins, lp)
        nested = any(o != lp and lp[0] <= o[0] and o[1] <= lp[1] for o in backward_loops(ins))
        if mix["v_mad_u64_u32"] >= 64 and not nested and any(op.startswith("ds_read") for op in mix):
            rows.append((lp, mix))
    assert rows, f"{kernel}: no radix-2^28 Montgomery row loop found"
    # 2 * C28 = 74 mads per CIOS step for C = 32: s28::mont_mul's row, one step per loop pass
    # (G = 1) or EFL_MONT28_UNROLL = 2 steps (148)
    def is_row(mix):
        return mix["v_mad_u64_u32"] in (74, 148)
    for lp, mix in rows:
        if is_row(mix):
            assert not any(op.startswith("scratch_") for op in mix), (kernel, lp, mix)
            assert mix["v_mad_u64_u32"] >= 0.7 * sum(mix.values()), (kernel, lp, mix)
    assert any(is_row(mix) for _, mix in rows), (kernel, [m for _, m in rows])
