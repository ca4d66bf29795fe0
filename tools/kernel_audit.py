#!/usr/bin/env python3
"""Per-kernel VGPR / AGPR / scratch / LDS usage from a ``-save-temps`` device assembly file
(``python -m llmctl.ops.build --save-temps`` writes build/ops/<src>-hip-amdgcn-amd-amdhsa-gfx950.s).

    python tools/kernel_audit.py build/ops/gemm64-hip-amdgcn-amd-amdhsa-gfx950.s [substring ...]
"""

import re
import sys


def audit(path, pats=()):
    s = open(path).read()
    rows = []
    for m in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", s, re.S):
        name, body = m.group(1), m.group(2)
        if pats and not any(p in name for p in pats):
            continue

        def f(k):
            r = re.search(rf"\.amdhsa_{k} (\d+)", body)
            return int(r.group(1)) if r else -1

        i = s.find(name + ":")
        j = s.find(".Lfunc_end", i)
        code = s[i:j]
        rows.append((name, f("next_free_vgpr"), f("accum_offset"), f("private_segment_fixed_size"),
                     f("group_segment_fixed_size"), code.count("scratch_store"), code.count("scratch_load")))
    for r in rows:
        print(f"{r[0][:90]:90s} vgpr {r[1]:3d} agpr@{r[2]:3d} scratch {r[3]:4d}B lds {r[4]:6d} "
              f"spill st/ld {r[5]}/{r[6]}")
    return rows


if __name__ == "__main__":
    audit(sys.argv[1], sys.argv[2:])
