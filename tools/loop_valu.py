#!/usr/bin/env python3
"""VALU count of one loop of a kernel's device assembly (tools/isa_stats.py --dump),
split into the always-executed path and the exec-masked regions (s_cbranch_execz X
... X:), which a wave runs only when some lane takes them (the pass re-scan, the
terminal-ply block).

    python tools/loop_valu.py /tmp/isa8/<kernel>.s            # the loop with the most VALU
    python tools/loop_valu.py /tmp/isa8/<kernel>.s --header 82
"""
import argparse
import re
import sys


def loops(lines):
    """header label -> (first line, last line) of each loop (from the '; =>This Loop Header' comments)."""
    res = {}
    for i, l in enumerate(lines):
        m = re.match(r"^\.LBB(\d+_\d+):.*Loop Header", l)
        if m:
            res[m.group(1)] = i
    out = {}
    for lab, start in res.items():
        end = max((i for i, l in enumerate(lines) if re.search(r"s_(c)?branch\w*\s+\.LBB%s\b" % lab, l)), default=start)
        out[lab] = (start, end)
    return out


def valu(lines, a, b):
    return sum(1 for l in lines[a:b] if re.match(r"\s+v_", l))


def salu(lines, a, b):
    return sum(1 for l in lines[a:b] if re.match(r"\s+s_", l) and not re.match(r"\s+s_(waitcnt|nop|cbranch|branch)", l))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--header")
    a = ap.parse_args()
    L = open(a.asm).read().split("\n")
    lp = loops(L)
    if a.header:
        key = next(k for k in lp if k.endswith("_" + a.header) or k == a.header)
    else:
        key = max(lp, key=lambda k: valu(L, *lp[k]))
    start, end = lp[key]
    regions, i = [], start
    while i < end:
        m = re.search(r"s_cbranch_execz (\.LBB\d+_\d+)", L[i])
        if m:
            j = i
            while not L[j].startswith(m.group(1) + ":"):
                j += 1
            regions.append((i, j))
            i = j
        i += 1
    tot = valu(L, start, end)
    cond = sum(valu(L, x, y) for x, y in regions)
    print("loop .LBB%s lines %d-%d: VALU %d, always %d, exec-masked regions %s; SALU %d" % (
        key, start, end, tot, tot - cond, [valu(L, x, y) for x, y in regions], salu(L, start, end)))


if __name__ == "__main__":
    sys.exit(main())
