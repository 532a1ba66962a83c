#!/usr/bin/env python3
"""Per-kernel instruction counts of a gfx950 device assembly file (hipcc
--cuda-device-only -S): VALU / SALU / LDS / spill-lane moves, SGPR/VGPR
counts and spills. Used to check the SOR kernels' register pressure after a
change (an SGPR spill is a v_writelane / v_readlane pair, i.e. VALU work).

usage: scripts/asm_stats.py file.s [name-substring]
"""
import re
import sys


def kernels(text):
    cur, body = None, []
    for line in text.splitlines():
        m = re.match(r"^(_Z\w+):", line)
        if m:
            cur, body = m.group(1), []
            continue
        if cur is not None:
            body.append(line)
            if "s_endpgm" in line:
                yield cur, body
                cur = None


def meta(text):
    out = {}
    for m in re.finditer(r"\.name:\s+(\S+)(.*?)(?=\n\s+- \.|\n\.\.\.|\Z)", text, re.S):
        blk = m.group(2)
        d = {}
        for key in ("sgpr_count", "sgpr_spill_count", "vgpr_count", "vgpr_spill_count", "private_segment_fixed_size"):
            k = re.search(r"\." + key + r":\s+(\d+)", blk)
            if k:
                d[key] = int(k.group(1))
        out[m.group(1)] = d
    return out


def main():
    text = open(sys.argv[1]).read()
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    md = meta(text)
    for name, body in kernels(text):
        if sub not in name:
            continue
        ins = [l.strip().split()[0] for l in body if l.startswith("\t") and not l.strip().startswith((";", "."))]
        c = lambda p: sum(1 for i in ins if i.startswith(p))
        print(name)
        print("  insts %d  v_* %d  s_* %d  ds_* %d  readlane %d  writelane %d  v_mov_b64 %d  dpp %d" % (
            len(ins), c("v_"), c("s_"), c("ds_"), c("v_readlane"), c("v_writelane"), c("v_mov_b64"),
            sum(1 for l in body if "_dpp" in l)))
        print("  " + "  ".join("%s %s" % kv for kv in md.get(name, {}).items()))


if __name__ == "__main__":
    main()
