#!/usr/bin/env python3
"""Instruction mix of the stencil kernel's steady-state loop (static count).

Reads the built per-depth code objects (as tools/loop_align.py does), finds the
steady-state loop of life_tb_kernel<K, RULE, NP, HAND> (the last loop with >= 32
8-byte instructions) and classifies its instructions.  One loop iteration is one
block of PF steps x K stages, so per stage-step (= one lane group, 64 columns x
one generation, per lane) the counts are divided by K * PF.  The VALU roofline of
bench.py prices the stage logic from this: full-rate v_bitop3 / logic ops take one
issue slot, DPP moves and v_alignbit (half rate on gfx950,
profiles/r01/valu_rate.json) two.

    python tools/valu_mix.py mpi-game-of-life_amd/libgol.so [--json out.json]
"""
import json
import re
import sys

import loop_align as la

HALF = ("v_alignbit", "_dpp", "v_and_or", "v_lshl_or", "v_add3")


def classify(mn):
    if mn.startswith("v_"):
        if "dpp" in mn or any(mn.startswith(h) for h in HALF if not h.startswith("_")):
            return "valu_half"
        return "valu_full"
    if mn.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if mn.startswith("s_"):
        return "salu"
    return "other"


def loop_body(body):
    base = int(body[0].split()[0], 16)
    ins = []
    for l in body:
        m = re.search(r"^\s*(\S+)(.*?)// ([0-9A-F]+): ([0-9A-F]{8})( [0-9A-F]{8})?", l)
        if m:
            ins.append((int(m.group(3), 16), 8 if m.group(5) else 4, m.group(1), l))
    loops = []
    for a, _, mn, l in ins:
        m = re.search(r"s_c?branch\w* .*\+0x([0-9a-f]+)>", l)
        if m and int(m.group(1), 16) + base < a:
            loops.append((int(m.group(1), 16) + base, a))
    cands = [(lo, hi, sum(1 for a, sz, _, _ in ins if lo <= a <= hi and sz == 8))
             for lo, hi in loops]
    cands = [c for c in cands if c[2] >= 32]
    if not cands:
        return None
    # the steady-state loop: of the innermost candidate loops, the one with the most
    # compute (the control flow may wrap bigger loops around it)
    inner = [c for c in cands
             if not any(d is not c and c[0] <= d[0] and d[1] <= c[1] for d in cands)]
    lo, hi, _ = max(inner, key=lambda c: c[2])
    return [(mn, l) for a, _, mn, l in ins if lo <= a <= hi]


def main():
    so = sys.argv[1]
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    lines, vg = la.disassemble(so)
    recs = []
    for i, l in enumerate(lines):
        m = la.KRE.match(l)
        if not m:
            continue
        K, rule, np_, hand, toff = (int(x) for x in m.groups())
        end = next(j for j in range(i + 1, len(lines)) if not lines[j].strip())
        body = loop_body(lines[i:end])
        if body is None:
            continue
        pf = 8 if (np_ == 2 and K >= 16) else 4
        cnt = {}
        bitop3 = dpp = align = 0
        for mn, _ in body:
            c = classify(mn)
            cnt[c] = cnt.get(c, 0) + 1
            bitop3 += mn.startswith("v_bitop3")
            dpp += "dpp" in mn
            align += mn.startswith("v_alignbit")
        steps = K * pf
        per = {k: round(v / steps, 3) for k, v in cnt.items()}
        slots = (cnt.get("valu_full", 0) + 2 * cnt.get("valu_half", 0)) / steps
        stage_slots = (bitop3 + 2 * (dpp + align)) / steps
        rec = {"K": K, "rule": rule, "np": np_, "hand": bool(hand), "toff": toff, "vgprs": vg.get((K, rule, np_, hand, toff)),
               "loop_instrs": len(body), "stage_steps_per_iter": steps,
               "per_stage_step": per, "v_bitop3": round(bitop3 / steps, 3),
               "dpp": round(dpp / steps, 3), "v_alignbit": round(align / steps, 3),
               "valu_slots_per_stage_step": round(slots, 3),
               "stage_logic_slots_per_stage_step": round(stage_slots, 3)}
        recs.append(rec)
        print(f"<{K:2d},{rule},{np_},{int(hand)},{toff}> per stage-step: bitop3 {rec['v_bitop3']:5.2f} "
              f"dpp {rec['dpp']:4.2f} alignbit {rec['v_alignbit']:4.2f} | all VALU slots "
              f"{slots:5.2f} (stage logic {stage_slots:5.2f}) | {per}")
    if out:
        json.dump({"source": "static disassembly of the steady-state loop, tools/valu_mix.py",
                   "slot_weights": {"full_rate": 1, "half_rate (DPP, v_alignbit)": 2},
                   "kernels": recs}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
