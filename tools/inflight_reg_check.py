#!/usr/bin/env python3
"""Linear-scan check of a kernel's ISA: no instruction other than the retiring s_waitcnt touches the
destination VGPRs of an outstanding register load (buffer_load / global_load without `lds`) --
the hazard of asm loads whose destinations the compiler thinks are already written.  vmcnt is
modelled in issue order (loads, LDS-DMA and stores count together); branches are read as fall-through.

    python tools/inflight_reg_check.py <device .s> <kernel-substring> [...]
"""
import re
import sys


def regs(tok):
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"v(\d+)", tok)
    return {int(m.group(1))} if m else set()


def check(path, pats):
    s = open(path).read()
    for name in re.findall(r"^(_Z\S+):[ \t]*(?:;.*)?$", s, re.M):
        if not any(p in name for p in pats):
            continue
        i = s.index(name + ":")
        j = s.find(".Lfunc_end", i)
        out = []  # outstanding vmem ops: set of dest regs (empty for DMA / stores)
        bad = 0
        for line in s[i:j].split("\n"):
            l = line.strip()
            if not l or l.startswith((";", ".")) or l.endswith(":"):
                continue
            op = l.split()[0]
            toks = [t for t in re.split(r"[,\s]+", l)[1:] if t]
            if op == "s_waitcnt":
                m = re.search(r"vmcnt\((\d+)\)", l)
                if m:
                    n = int(m.group(1))
                    while len(out) > n:
                        out.pop(0)
                continue
            if op.startswith(("buffer_load", "global_load", "scratch_load", "buffer_store", "global_store",
                              "scratch_store", "buffer_atomic", "global_atomic")):
                dst = regs(toks[0]) if ("load" in op and "lds" not in l) else set()
                # a VMEM op reading an in-flight load's destination as an address / data is a hazard too
                src = set()
                for t in toks[1 if dst else 0:]:
                    src |= regs(t)
                pend = set().union(*out) if out else set()
                if (src | dst) & pend:
                    bad += 1
                    if bad <= 5:
                        print("   ", l[:100])
                out.append(dst)
                continue
            if op.startswith("s_"):
                continue
            used = set()
            for t in toks:
                used |= regs(t)
            pend = set().union(*out) if out else set()
            if used & pend:
                bad += 1
                if bad <= 5:
                    print("   ", l[:100], sorted(used & pend)[:4])
        print(f"{name[:90]}: {bad} touches of in-flight load destinations")


if __name__ == "__main__":
    check(sys.argv[1], sys.argv[2:])
