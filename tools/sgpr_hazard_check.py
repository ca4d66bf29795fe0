#!/usr/bin/env python3
"""Flag VALU writes of SGPRs (v_readlane / v_readfirstlane) read by a VMEM instruction fewer than
5 wait states later -- the hazard hipcc does not pad when the VMEM instruction sits in inline asm
(the LDS-DMA buffer_loads of the GEMM / attention kernels).

    python tools/sgpr_hazard_check.py <device .s> [kernel-substring ...]
"""
import re
import sys


def sregs(tok):
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"s(\d+)", tok)
    return {int(m.group(1))} if m else set()


def check(path, pats):
    s = open(path).read()
    names = re.findall(r"^(_Z\S+):\s*$", s, re.M)
    total = 0
    for n in names:
        if pats and not any(p in n for p in pats):
            continue
        i = s.index(n + ":")
        j = s.find(".Lfunc_end", i)
        lines = [l.strip() for l in s[i:j].split("\n")]
        ins = [l for l in lines if l and not l.startswith((";", ".", "//")) and not l.endswith(":")]
        hits = 0
        for k, l in enumerate(ins):
            op = l.split()[0]
            if op not in ("v_readlane_b32", "v_readfirstlane_b32"):
                continue
            dst = sregs(l.split()[1].rstrip(","))
            ws = 0
            for l2 in ins[k + 1:k + 12]:
                op2 = l2.split()[0]
                if op2.startswith(("buffer_", "global_", "scratch_")):
                    used = set()
                    for tok in re.split(r"[,\s]+", l2)[1:]:
                        used |= sregs(tok)
                    if used & dst and ws < 5:
                        hits += 1
                        print(f"  {n[:70]}: '{l}' -> {ws} wait states -> '{l2}'")
                ws += int(op2 == "s_nop" and l2.split()[1] or 0) + 1 if op2 == "s_nop" else 1
        total += hits
    print("hazards:", total)
    return total


if __name__ == "__main__":
    check(sys.argv[1], sys.argv[2:])
