"""CPU check of the built library's gfx950 code (no GPU): the pipelined
gathering kernel's counted wait (linearize_gather_kernel, m3s_gn.hip) is only
correct if at least NPL vector-memory operations follow the 8 LDS-DMA refill
loads on every path back to the loop top's `s_waitcnt vmcnt(NPL)` (vmcnt counts
in issue order; the inline-asm LDS reads of the slot are invisible to the
compiler's own waits). The compiler could sink, split or merge the plane
stores that follow the refill; this test disassembles the code object in
libm3s_gn.so and checks every branch to, and every fall-through into, such a
wait."""
import os
import re
import shutil
import struct
import subprocess

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
LIB = os.path.join(ROOT, "mast3r-slam-ysh_amd", "mast3r_slam_backends", "libm3s_gn.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
NPL = {0: 4, 1: 4, 2: 3}  # planes per mode: points, rays, calib (PixIn<MODE>::kPlanes)


def code_object(path):
    data = open(path, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    i = data.find(magic)
    assert i >= 0, "no offload bundle in the library"
    n = struct.unpack_from("<Q", data, i + 24)[0]
    off = i + 32
    for _ in range(n):
        o, sz, tl = struct.unpack_from("<QQQ", data, off)
        trip = data[off + 24:off + 24 + tl].decode()
        off += 24 + tl
        if "gfx950" in trip:
            return data[i + o:i + o + sz]
    raise AssertionError("no gfx950 code object")


@pytest.fixture(scope="module")
def disasm(tmp_path_factory):
    if not (os.path.exists(LIB) and os.path.exists(OBJDUMP)):
        pytest.skip("library or llvm-objdump missing")
    co = tmp_path_factory.mktemp("isa") / "gn.co"
    co.write_bytes(code_object(LIB))
    return subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", str(co)], check=True, capture_output=True,
                          text=True).stdout


def kernel_insns(text, mode):
    """[(address, instruction)] of linearize_gather_kernel<mode>."""
    name = f"linearize_gather_kernelILi{mode}EEEvNS_7LinArgsE>:"
    lines = text.splitlines()
    start = next(i for i, l in enumerate(lines) if l.endswith(name))
    out = []
    for l in lines[start + 1:]:
        if re.match(r"^[0-9a-f]+ <", l):
            break
        m = re.search(r"//\s*([0-9A-Fa-f]+):?", l)
        if m and l.strip():
            out.append((int(m.group(1), 16), l.split("//")[0].strip()))
    return out


VMEM = re.compile(r"^(global|buffer|flat)_(load|store|atomic)")


@pytest.mark.parametrize("mode", [1, 2])
def test_gather_refill_is_covered_by_counted_wait(disasm, mode):
    ins = kernel_insns(disasm, mode)
    npl = NPL[mode]
    addr_idx = {a: i for i, (a, _) in enumerate(ins)}
    waits = [i for i, (_, t) in enumerate(ins) if t == f"s_waitcnt vmcnt({npl})"]
    assert waits, "the loop top's counted wait is missing"
    lds = [i for i, (_, t) in enumerate(ins) if VMEM.match(t) and t.endswith(" lds")]
    assert lds, "no LDS-DMA refill found"

    def vmem_after_last_refill(end):  # scanning back from instruction `end` (exclusive)
        n = 0
        for j in range(end - 1, -1, -1):
            t = ins[j][1]
            if VMEM.match(t):
                if t.endswith(" lds"):
                    return n
                n += 1
            if t.startswith("s_endpgm"):
                return None
        return None

    checked = 0
    for w in waits:
        wa = ins[w][0]
        # branches landing at the wait (or on the instructions right before it
        # in the same block: s_waitcnt lgkmcnt / s_nop / moves)
        for j, (a, t) in enumerate(ins):
            m = re.match(r"^s_(c?branch\w*)\s", t)
            if not m:
                continue
            tgt = re.search(r"<[^+]+\+0x([0-9a-f]+)>", disasm_line(disasm, a))
            if not tgt:
                continue
            base = ins[0][0] - 0x0  # the function's first instruction address
            ta = kernel_base(disasm, mode) + int(tgt.group(1), 16)
            if ta in addr_idx and addr_idx[ta] <= w and all(not VMEM.match(ins[q][1]) and not ins[q][1].startswith("s_c")
                                                          for q in range(addr_idx[ta], w)):
                n = vmem_after_last_refill(j)
                if n is not None:
                    assert n >= npl, (mode, hex(a), n)
                    checked += 1
        # fall-through into the wait
        if w > 0 and not ins[w - 1][1].startswith("s_branch"):
            n = vmem_after_last_refill(w)
            if n is not None:
                assert n >= npl, (mode, hex(wa), n)
                checked += 1
    print(f"mode {mode}: {checked} paths into the counted wait checked")
    assert checked >= 1


_LINES = {}


def disasm_line(text, addr):
    if not _LINES:
        for l in text.splitlines():
            m = re.search(r"//\s*([0-9A-Fa-f]+):?", l)
            if m:
                _LINES[int(m.group(1), 16)] = l
    return _LINES.get(addr, "")


def kernel_base(text, mode):
    name = f"linearize_gather_kernelILi{mode}EEEvNS_7LinArgsE>:"
    for l in text.splitlines():
        if l.endswith(name):
            return int(l.split()[0], 16)
    raise AssertionError(name)
