#!/usr/bin/env python3
"""Scan a gfx950 .s for VMEM instructions whose scalar operands (buffer resource / soffset) were
written by a VALU (v_readlane / v_readfirstlane / v_cmp...) fewer than 5 instructions earlier —
the "VALU writes SGPR -> VMEM reads it" hazard that hipcc does not pad inside inline asm.

    asm_hazard_scan.py file.s [kernel-substring]"""
import re
import sys


def sregs(tok):
    m = re.match(r"s\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"s(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def main():
    txt = open(sys.argv[1]).read()
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    for fm in re.finditer(r"^(_Z\S+):", txt, re.M):
        name = fm.group(1)
        if want not in name:
            continue
        end = txt.find(".Lfunc_end", fm.end())
        lines = [l.strip() for l in txt[fm.end():end].split("\n")]
        ins = [l for l in lines if l and not l.startswith((";", ".")) and not l.endswith(":")]
        hits = 0
        for i, l in enumerate(ins):
            if not re.match(r"(buffer_|global_load_lds|s_load|s_buffer)", l):
                continue
            ops = re.split(r"[\s,]+", l)
            used = set()
            for t in ops[1:]:
                used |= sregs(t)
            for j in range(max(0, i - 5), i):
                p = ins[j]
                if p.startswith("s_nop"):
                    n = int(re.findall(r"\d+", p)[0]) + 1
                    if n >= 5:
                        break
                    continue
                if re.match(r"v_(readlane|readfirstlane|cmp|add_co|sub_co|div_scale)", p):
                    dst = sregs(re.split(r"[\s,]+", p)[1])
                    if dst & used:
                        hits += 1
                        if hits <= 12:
                            print(f"{name[:60]}: {p}  ->  {l}   (distance {i - j})")
        print(f"{name[:70]}: {hits} hazards")


if __name__ == "__main__":
    main()
