#!/usr/bin/env python3
"""Code placement of the stencil kernel's steady-state loop.

On gfx950 the hot loop of life_tb_kernel (DPP move, v_alignbit, v_bitop3 chains,
all 8-byte encodings) issues 10-25% faster at addresses = 4 mod 8 when 2+ waves
share a SIMD, and faster at 0 mod 8 with one wave (K >= 20): builds with
identical instructions and register allocation differ only in that placement
(profiles/r01/loop_alignment_ab.jsonl, tools/valu_rate.hip "mix_at_*").
life_kernels.hip aligns the compute of each steady-state block to 8 bytes and
adds a 4-byte s_nop when csrc/loop_place.h says so.  This tool reads the built
libgol.so, reports per life_tb_kernel<K, RULE, NP, HAND, TOFF> the share of the main
loop's 8-byte instructions at the wanted parity (4 mod 8 when the kernel's
registers admit 2+ waves per SIMD, from the code object's .vgpr_count), and
with --update flips the pad of misplaced kernels in loop_place.h (rebuild
afterwards; a kernel's code does not depend on the other kernels').  Exit
status 1 if a B/S2 or B3/S23 kernel at depth >= 8 is misplaced.

    python tools/loop_align.py mpi-game-of-life_amd/libgol.so [--update]
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
HERE = os.path.dirname(os.path.abspath(__file__))
HEADER = os.path.join(HERE, "..", "mpi-game-of-life_amd", "csrc", "loop_place.h")
# life_tb_kernel<K, RULE, NP, HAND, TOFF, MP> (MP, r05: the multi-pass form)
KRE = re.compile(r"^[0-9a-f]+ <_ZN3gol12_GLOBAL__N_114life_tb_kernelILi(\d+)ELi(\d+)ELi(\d+)ELb(\d)ELi(\d+)ELb(\d)EEEvNS_8StepArgsE>:")
NRE = re.compile(r"life_tb_kernelILi(\d+)ELi(\d+)ELi(\d+)ELb(\d)ELi(\d+)ELb(\d)EEEvNS_8StepArgsE")


def disassemble_one(obj):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat"), os.path.join(d, "co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj,
                        os.path.join(d, "junk")], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}",
                        f"--output={co}"], check=True)
        dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], check=True,
                             capture_output=True, text=True).stdout.split("\n")
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True,
                               capture_output=True, text=True).stdout
        return dis, vgpr_counts(notes)


def disassemble(so):
    """The stencil kernels live in one code object per depth: read the per-depth
    objects the library was linked from (build/ next to it)."""
    objs = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(so)), "build",
                                         "life_tb_d*.o")))
    dis, vg = [], {}
    for o in objs or [so]:
        d, v = disassemble_one(o)
        dis += d + [""]
        vg.update(v)
    return dis, vg


def vgpr_counts(notes):
    """{(K, RULE, NP, HAND, TOFF): .vgpr_count} of the stencil kernels, from the code
    object metadata (gfx950: one unified register file, 512 per SIMD lane)."""
    out, name, vg = {}, None, None
    for l in notes.split("\n") + ["- end"]:
        s = l.strip()
        if s.startswith("- "):  # a new metadata entry: flush the previous one
            if name and vg is not None:
                out[name] = vg
            name, vg = None, None
            s = s[2:]
        if s.startswith(".name:"):
            m = NRE.search(s)
            name = tuple(int(x) for x in m.groups()) if m else None
        elif s.startswith(".vgpr_count:"):
            vg = int(s.split(":")[1])
    return out


def main_loop_fractions(body, births):
    """[(mask, fraction of the loop's 8-byte instructions at 4 mod 8, count)] for the
    steady-state loops: one for B/S2 kernels; for kernels with births (r04) the
    loop without the births mask (mask 0: the smaller one) and the masked loop
    (mask 1: the bigger ones, kPureMask and a hand-off consumer's kSide blocks),
    which get their own pad."""
    base = int(body[0].split()[0], 16)
    ins = []
    for l in body:
        m = re.search(r"// ([0-9A-F]+): ([0-9A-F]{8})( [0-9A-F]{8})?", l)
        if m:
            ins.append((int(m.group(1), 16), 8 if m.group(3) else 4, l))
    loops = []
    for a, _, l in ins:
        m = re.search(r"s_c?branch\w* .*\+0x([0-9a-f]+)>", l)
        if m and int(m.group(1), 16) + base < a:
            loops.append((int(m.group(1), 16) + base, a))
    cands = []
    for lo, hi in loops:
        eight = [a for a, sz, _ in ins if lo <= a <= hi and sz == 8]
        if len(eight) >= 32:
            cands.append((lo, hi, eight))
    if not cands:
        return []
    # the steady-state loops: innermost candidates with the most compute (the
    # control flow may wrap bigger loops around them; a hand-off kernel's flag
    # polls split its blocks into several backward branches of about one size)
    inner = [c for c in cands
             if not any(d is not c and c[0] <= d[0] and d[1] <= c[1] for d in cands)]
    top = max(len(c[2]) for c in inner)
    big = [c for c in inner if len(c[2]) >= 0.8 * top]
    frac = lambda e8: sum(1 for a in e8 if a % 8 == 4) / len(e8)
    if not births:
        # the pure loop: the smallest (r05: a hand-off consumer's last blocks, with
        # the per-load side-row selects and the multi-pass checks, form bigger loops)
        lo, hi, e8 = min(big, key=lambda c: len(c[2]))
        return [(0, frac(e8), len(e8))]
    small = min(len(c[2]) for c in big)
    out = []
    for mask, grp in ((0, [c for c in big if len(c[2]) <= 1.04 * small]),
                      (1, [c for c in big if len(c[2]) > 1.04 * small])):
        if grp:
            fr = [frac(c[2]) for c in grp]
            # the worst-placed copy, unless some copy has 4-byte code inside (~50%)
            f = min(fr) if all(x >= 0.5 for x in fr) or all(x < 0.5 for x in fr) else min(fr)
            out.append((mask, f, len(grp[0][2])))
    return out


def current_pads():
    pads = set()
    if os.path.exists(HEADER):
        for m in re.finditer(r"\{(\d+), (\d+), (\d+), (\d+), (\d+), (\d+)\}", open(HEADER).read()):
            if m.group(1) != "0":
                pads.add(tuple(int(x) for x in m.groups()))
    return pads


def write_header(pads):
    rows = "".join(f"    {{{k}, {r}, {n}, {h}, {t}, {mk}}},\n" for k, r, n, h, t, mk in sorted(pads))
    open(HEADER, "w").write(f"""// loop_place.h -- GENERATED by tools/loop_align.py --update from the built
// libgol.so; do not edit by hand.  life_loop_pad(K, RULE, NP, HAND, TOFF, MASK) = 1
// adds a 4-byte s_nop after the 8-byte alignment before the compute of each
// steady-state block of life_tb_kernel<K, RULE, NP, HAND, TOFF, MP> without (MASK
// bit 0 clear) or with (bit 0 set) the births mask, MASK bit 1 = MP (the
// multi-pass form; see life_stencil.h).
#pragma once

namespace gol {{

struct LoopPad {{
    int K, rule, np, hand, toff, mask;
}};
constexpr LoopPad kLoopPads[] = {{
{rows}    {{0, 0, 0, 0, 0, 0}}  // end
}};

constexpr int life_loop_pad(int K, int RULE, int NP, bool HAND, int TOFF, int MASK)
{{
    for (const LoopPad& p : kLoopPads)
        if (p.K == K && p.rule == RULE && p.np == NP && p.hand == (HAND ? 1 : 0) && p.toff == TOFF &&
            p.mask == MASK)
            return 1;
    return 0;
}}

}}  // namespace gol
""")


def main():
    if sys.argv[1] == "--init":  # empty table (no pads)
        write_header(set())
        return 0
    so = sys.argv[1]
    update = "--update" in sys.argv
    lines, vgprs = disassemble(so)
    pads = current_pads()
    new = set(pads)
    bad = 0
    for i, l in enumerate(lines):
        m = KRE.match(l)
        if not m:
            continue
        key = tuple(int(x) for x in m.groups())
        mp, key = key[5], key[:5]
        end = next(j for j in range(i + 1, len(lines)) if not lines[j].strip())
        # 2+ waves per SIMD when the kernel fits 256 registers (512 per SIMD lane)
        want4 = vgprs.get(key + (mp,), 0) <= 256 if vgprs else key[0] < 20
        for mask, frac, n in main_loop_fractions(lines[i:end], key[1] != 0):
            kmask = key + (mask | (mp << 1),)
            good = frac if want4 else 1.0 - frac
            hot = key[1] in (0, 1) and key[0] >= 8
            ok = good >= 0.9
            print(f"life_tb_kernel<{key[0]:2d}, {key[1]}, {key[2]}, {bool(key[3])}, {key[4]}{', MP' if mp else ''}> "
                  f"{'masked' if mask else 'plain '} ({vgprs.get(key + (mp,), '?')} regs): {n:5d} 8-byte instrs, "
                  f"{100 * good:3.0f}% at {'4' if want4 else '0'} mod 8, pad {int(kmask in pads)}"
                  f"{'' if ok else '  <- misplaced'}")
            if good < 0.35:  # a clear miss; ~50% means 4-byte code inside the compute
                new ^= {kmask}
            bad += int(hot and not ok)
    if update and new != pads:
        write_header(new)
        print(f"updated {HEADER}: {len(new)} padded kernels; rebuild")
    print(f"{bad} hot kernels misplaced")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
