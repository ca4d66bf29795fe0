#!/usr/bin/env python3
"""Check that no instruction touches the destination register of an inline-asm VMEM load before
the counted wait that retires it (a hipcc register copy of an in-flight asm load destination is a
silent data race; round 3 found one in the persistent dK/dV kernel).

    asm_inflight_scan.py file.s <kernel-substring> <load-regex> <retire-vmcnt> [--waits N]

<load-regex> matches the asm loads to follow (e.g. 'buffer_load_dword (v\\d+), v\\d+, s\\[\\d+:\\d+\\], 0 offen nt$');
a load counts as retired at the N-th ``s_waitcnt vmcnt(<retire-vmcnt>)`` after it (or any vmcnt(0)).
Example (gemm64 side job, SIDE=1: L(t) is retired by the j = 3 wait of tile t+1, vmcnt(11)):

    hipcc ... --offload-device-only -S gemm64.hip -o g64.s
    asm_inflight_scan.py g64.s 'gemm64_kernelILb1ELb1ELi0ELi4ELi1ELi1E' \\
        'buffer_load_dword (v\\d+), v\\d+, s\\[\\d+:\\d+\\], 0 offen nt$' 11 --waits 2
"""
import argparse
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("load_regex")
    ap.add_argument("retire_vmcnt", type=int)
    ap.add_argument("--waits", type=int, default=1)
    a = ap.parse_args()
    txt = open(a.asm).read()
    pat = re.compile(a.load_regex)
    total_bad = 0
    for fm in re.finditer(r"^(_Z\S+):", txt, re.M):
        name = fm.group(1)
        if a.kernel not in name:
            continue
        end = txt.find(".Lfunc_end", fm.end())
        ins = [l.split(";")[0].strip() for l in txt[fm.end():end].split("\n")]
        ins = [l for l in ins if l and not l.startswith(".") and not l.endswith(":")]
        loads = bad = 0
        for i, l in enumerate(ins):
            m = pat.match(l)
            if not m:
                continue
            loads += 1
            reg, waits = m.group(1), 0
            for t in ins[i + 1:]:
                w = re.match(r"s_waitcnt vmcnt\((\d+)\)", t)
                if w:
                    n = int(w.group(1))
                    if n == 0:
                        break
                    if n == a.retire_vmcnt:
                        waits += 1
                        if waits >= a.waits:
                            break
                if re.search(r"\b%s\b" % re.escape(reg), t):
                    bad += 1
                    print(f"{name[:60]}: {reg} used before its retiring wait: {t}")
                    break
        print(f"{name[:80]}: {loads} loads, {bad} early uses")
        total_bad += bad
    raise SystemExit(1 if total_bad else 0)


if __name__ == "__main__":
    main()
