#!/usr/bin/env python3
"""List the global stores of source_kernel_ifelse with their basic block and
the exec-mask operations on the path into that block (gfx950 ISA)."""
import re
import sys

L = open(sys.argv[1]).read().split("\n")
st = next(i for i, l in enumerate(L) if l.startswith("_ZN3cfd20source_kernel_ifelse"))
end = next(i for i in range(st, len(L)) if L[i].startswith(".Lfunc_end"))
block = "entry"
for i in range(st, end):
    l = L[i].rstrip()
    m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):", l)
    if m:
        block = m.group(1)
        continue
    t = l.strip()
    if re.match(r"(s_and_saveexec|s_or_b64 exec|s_andn2_b64 exec|s_mov_b64 exec|s_xor_b64 exec|s_cbranch_exec)", t):
        print(f"{i - st:5d} {block:14s} {t}")
    if t.startswith("global_store"):
        print(f"{i - st:5d} {block:14s} {t}    <-- store")
