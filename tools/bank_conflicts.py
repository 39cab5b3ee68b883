#!/usr/bin/env python3
"""Dev tool: count VGPR bank conflicts (sources of one VALU instruction in the
same bank, bank = vgpr index mod 4) in the steady-state loop of a kernel in an
llvm-objdump disassembly.  Usage: bank_conflicts.py kernel.dis KERNEL_SUBSTR"""
import collections
import re
import sys


def main():
    lines = open(sys.argv[1]).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^[0-9a-f]+ <.*" + sys.argv[2], l))
    end = next(i for i in range(start + 1, len(lines)) if not lines[i].strip())
    body = lines[start:end]
    base = int(body[0].split()[0], 16)
    addr = lambda l: (int(m.group(1), 16) if (m := re.search(r"// ([0-9A-F]+):", l)) else None)
    loops = []
    for l in body:
        m = re.search(r"s_c?branch\w* .*\+0x([0-9a-f]+)>", l)
        if m and addr(l) is not None and int(m.group(1), 16) + base < addr(l):
            loops.append((int(m.group(1), 16) + base, addr(l)))
    lo, hi = max(loops, key=lambda a: a[1] - a[0])
    stats = collections.Counter()
    for l in body:
        a = addr(l)
        if a is None or not (lo <= a <= hi):
            continue
        ins = l.split("//")[0].strip()
        op = ins.split()[0]
        if not op.startswith("v_"):
            continue
        regs = re.findall(r"\bv(\d+)\b", ins)
        srcs = [int(r) for r in regs[1:]]  # first vgpr is the destination
        uniq = sorted(set(srcs))
        banks = collections.Counter(r % 4 for r in uniq)
        worst = max(banks.values()) if banks else 0
        stats[(op, len(uniq), worst)] += 1
    tot = sum(v for (op, n, w), v in stats.items() if w >= 2)
    print(f"loop {hex(lo - base)}..{hex(hi - base)}: VALU with >=2 distinct sources in one bank: {tot}")
    for k, v in sorted(stats.items(), key=lambda kv: -kv[1])[:12]:
        print(" ", k, v)


if __name__ == "__main__":
    main()
