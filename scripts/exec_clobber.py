#!/usr/bin/env python3
"""Heuristic check for a saved EXEC mask being overwritten before it is restored (round 6 debug aid).

In a gfx9 assembly listing, a divergent `if` saves EXEC (`s_mov_b64 s[a:b], exec` or
`s_and_saveexec_b64 s[a:b], ...`) and restores it at the join (`s_or_b64 exec, exec, s[a:b]`). If an
instruction between the two writes s[a] or s[a+1], the lanes masked off inside the `if` never come back.
This scans one function linearly (labels ignored): for every restore it finds the nearest preceding save
of the same pair and reports instructions in between that write either register.

usage: python scripts/exec_clobber.py FILE.s MANGLED_NAME_SUBSTRING
"""
import re
import sys


def sregs(tok: str) -> set:
    tok = tok.strip()
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"s(\d+)", tok)
    return {int(m.group(1))} if m else set()


def main(path: str, fn: str) -> int:
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*" + re.escape(fn) + r"\w*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    insts = []
    for i in range(start + 1, end):
        s = lines[i].split(";")[0].strip()
        if not s or s.startswith(".") or s.endswith(":"):
            continue
        insts.append((i, s))
    bad = 0
    for k, (i, s) in enumerate(insts):
        m = re.match(r"s_or_b64\s+exec,\s*exec,\s*(s\[\d+:\d+\])", s)
        if not m:
            continue
        saved = sregs(m.group(1))
        j = k - 1
        while j >= 0:
            sj = insts[j][1]
            if re.match(r"s_mov_b64\s+" + re.escape(m.group(1)) + r",\s*exec\b", sj) or \
               re.match(r"s_and_saveexec_b64\s+" + re.escape(m.group(1)) + r",", sj):
                break
            j -= 1
        if j < 0:
            continue
        for _, sj in insts[j + 1:k]:
            parts = sj.split(None, 1)
            if len(parts) < 2 or parts[0].startswith(("s_cbranch", "s_branch", "s_waitcnt", "s_nop", "buffer_", "global_store",
                                                      "ds_write", "scratch_store", "s_barrier")):
                continue
            dst = parts[1].split(",")[0]
            if sregs(dst) & saved:
                print(f"line {i + 1}: restore of {m.group(1)} (saved at line {insts[j][0] + 1}) after a write: {sj}")
                bad += 1
                break
    print(f"{bad} suspicious restores")
    return bad


if __name__ == "__main__":
    sys.exit(1 if main(sys.argv[1], sys.argv[2]) else 0)
