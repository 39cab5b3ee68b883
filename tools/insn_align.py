#!/usr/bin/env python3
"""Dev tool: alignment of the 8-byte (VOP3) instructions inside the loops of a
kernel, from llvm-objdump output.  Usage: insn_align.py file.dis KERNEL_SUBSTR"""
import re
import sys


def main():
    lines = open(sys.argv[1]).read().split("\n")
    s = next(i for i, l in enumerate(lines) if re.match(r"^[0-9a-f]+ <.*" + sys.argv[2], l))
    e = next(i for i in range(s + 1, len(lines)) if not lines[i].strip())
    body = lines[s:e]
    base = int(body[0].split()[0], 16)
    ins = []
    for l in body:
        m = re.search(r"// ([0-9A-F]+): ([0-9A-F]{8})( [0-9A-F]{8})?", l)
        if m:
            ins.append((int(m.group(1), 16), 8 if m.group(3) else 4, l))
    loops = []
    for a, sz, l in ins:
        m = re.search(r"s_c?branch\w* .*\+0x([0-9a-f]+)>", l)
        if m and int(m.group(1), 16) + base < a:
            loops.append((int(m.group(1), 16) + base, a))
    for lo, hi in sorted(set(loops)):
        eight = [a for a, sz, l in ins if lo <= a <= hi and sz == 8]
        odd = sum(1 for a in eight if a % 8 == 4)
        print(f"loop +{lo - base:#x}..+{hi - base:#x}: {len(eight)} 8-byte instrs, "
              f"{odd} at 4 mod 8 ({100.0 * odd / max(1, len(eight)):.0f}%)")


if __name__ == "__main__":
    main()
