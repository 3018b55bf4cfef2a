"""Instruction mix of a kernel's loops, from a hipcc -S device assembly.

usage: python tools/isa_loop.py file.s name-substring [--all]

A loop is a backward branch inside the kernel's body (label L, later a
branch to L); its body is every instruction between the label and the branch.
For each loop (innermost first, largest body last) it prints the count of VALU
(`v_`, packed-f32 `v_pk_` counted apart), SALU (`s_`), LDS (`ds_`), vector
memory (`buffer_` / `global_`) and waits, so that VALU per trip of the
linearize kernels' main loops can be read off an ISA.
Without --all only the loop with the most VALU is printed.
"""
import re
import sys
from collections import Counter


def kernel_body(text, sub):
    names = re.findall(r"^(\S+):\s*(?:;.*)?$", text, re.M)
    cand = [n for n in names if sub in n and not n.startswith(".")]
    if not cand:
        raise SystemExit(f"no symbol containing {sub!r}")
    name = cand[0]
    start = text.index(f"\n{name}:") + 1
    end = text.find("\n.Lfunc_end", start)
    return name, text[start:end].splitlines()


def classify(op):
    if op.startswith("v_pk_"):
        return "valu_pk"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    return "other"


def main():
    path, sub = sys.argv[1], sys.argv[2]
    show_all = "--all" in sys.argv
    name, lines = kernel_body(open(path).read(), sub)
    labels = {}
    insts = []  # (index, opcode, text)
    for ln in lines:
        s = ln.strip()
        m = re.match(r"^(\.LBB\S+):", s)
        if m:
            labels[m.group(1)] = len(insts)
            continue
        if not s or s.startswith((";", ".")):
            continue
        insts.append(s.split()[0])
        if insts[-1].startswith("s_cbranch") or insts[-1] == "s_branch":
            tgt = s.split()[-1]
            insts[-1] = (insts[-1], tgt)
    loops = []
    for i, op in enumerate(insts):
        if isinstance(op, tuple) and op[1] in labels and labels[op[1]] <= i:
            body = insts[labels[op[1]]:i + 1]
            c = Counter(classify(o[0] if isinstance(o, tuple) else o) for o in body)
            loops.append((op[1], len(body), c))
    if not loops:
        raise SystemExit(f"{name}: no loops")
    print(name)
    if not show_all:
        loops = [max(loops, key=lambda l: l[2]["valu"] + l[2]["valu_pk"])]
    for lab, n, c in loops:
        print(f"  loop {lab}: {n} instructions; VALU {c['valu'] + c['valu_pk']} "
              f"(v_pk_ {c['valu_pk']}), SALU {c['salu']}, LDS {c['lds']}, VMEM {c['vmem']}, "
              f"waits {c['wait']}, other {c['other']}")


if __name__ == "__main__":
    main()
