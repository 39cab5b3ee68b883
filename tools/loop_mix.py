#!/usr/bin/env python3
"""Dev tool: instruction mix of the innermost steady-state loop of a kernel in
an assembly file (hipcc -S output).  Finds backward branches and reports the
biggest loop body's instruction counts by opcode.

    python tools/loop_mix.py life_kernels.s 'life_tb_kernelILi8ELi0ELi0E'
"""
import collections
import re
import sys


def kernel_text(path, pat):
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^_Z\S*" + pat + r"\S*:", l):
            start = i
        elif start is not None and l.startswith(".Lfunc_end"):
            return lines[start:i]
    raise SystemExit("kernel not found")


def main():
    body = kernel_text(sys.argv[1], sys.argv[2])
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = i
    loops = []
    for i, l in enumerate(body):
        m = re.match(r"^\s+s_(cbranch_\w+|branch)\s+(\.LBB\w+)", l)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            loops.append((labels[m.group(2)], i))
    # innermost loops (containing no other loop), biggest first
    inner = [a for a in loops if not any(b != a and a[0] <= b[0] and b[1] <= a[1] for b in loops)]
    lo, hi = max(inner, key=lambda a: a[1] - a[0])
    cnt = collections.Counter()
    for l in body[lo:hi + 1]:
        l = l.strip()
        if not l or l.startswith((";", ".")):
            continue
        op = l.split()[0]
        if "dpp" in l or "row_" in l or "wave_sh" in l:
            op += "(dpp)"
        cnt[op] += 1
    tot = sum(cnt.values())
    valu = sum(v for k, v in cnt.items() if k.startswith("v_"))
    print(f"loop lines {lo}-{hi}: {tot} instructions, {valu} VALU")
    for k, v in cnt.most_common():
        print(f"  {v:6d} {k}")


if __name__ == "__main__":
    main()
