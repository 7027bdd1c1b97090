#!/usr/bin/env python3
"""Attribute a kernel's spill / scratch instructions to source lines.

Input: a gfx950 assembly file compiled with `-S -gline-tables-only --cuda-device-only`.
For one function (mangled-name substring) it counts scratch loads/stores, SGPR-spill lane moves
(v_writelane / v_readlane) and reports the source lines (.loc) they sit under, most first.

  hipcc -O3 -gline-tables-only -S --cuda-device-only ... tsw_plan.hip -o plan.s
  python scripts/isa_scratch.py plan.s k_planILb1ELb1ELb1ELb0E
"""
from __future__ import annotations

import collections
import re
import sys


def parse(path: str, fn: str, top: int = 30) -> dict:
    files: dict[int, str] = {}
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        m = re.match(r"\s*\.file\s+(\d+)\s+\"[^\"]*\"\s+\"([^\"]+)\"", l)
        if m:
            files[int(m.group(1))] = m.group(2)
        if start is None and re.match(r"^_Z\w*" + re.escape(fn) + r"\w*:", l):
            start = i
    if start is None:
        raise SystemExit(f"function matching {fn!r} not found")
    kinds = ("scratch_load", "scratch_store", "v_writelane", "v_readlane", "s_barrier", "global_load",
             "global_store", "ds_", "flat_")
    tot: collections.Counter = collections.Counter()
    per_line: dict[str, collections.Counter] = collections.defaultdict(collections.Counter)
    loc = "?"
    for l in lines[start + 1:]:
        s = l.strip()
        if s.startswith(".Lfunc_end"):
            break
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if m:
            loc = f"{files.get(int(m.group(1)), m.group(1))}:{m.group(2)}"
            continue
        if not s or s[0] in ".;" or s.endswith(":"):
            continue
        op = s.split()[0]
        tot["insts"] += 1
        for k in kinds:
            if op.startswith(k):
                tot[k] += 1
                per_line[loc][k] += 1
    spill = lambda c: c["scratch_load"] + c["scratch_store"]  # noqa: E731
    ranked = sorted(per_line.items(), key=lambda kv: -spill(kv[1]))
    return {"totals": dict(tot),
            "scratch_by_line": [(k, dict(v)) for k, v in ranked[:top] if spill(v)],
            "lanes_by_line": [(k, dict(v)) for k, v in sorted(per_line.items(),
                              key=lambda kv: -(kv[1]["v_writelane"] + kv[1]["v_readlane"]))[:top]
                              if v["v_writelane"] + v["v_readlane"]]}


if __name__ == "__main__":
    r = parse(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 30)
    print("totals", r["totals"])
    print("-- scratch ops by source line")
    for k, v in r["scratch_by_line"]:
        print(f"  {k:28s} {v}")
    print("-- SGPR-spill lane moves by source line")
    for k, v in r["lanes_by_line"]:
        print(f"  {k:28s} {v}")


def per_line_mix(path: str, fn: str, src: str, lo: int, hi: int) -> dict:
    """Static instruction mix (valu / salu / ds / vmem / lane moves) per source line of `src` in [lo, hi]
    for the function matching `fn` (a loop body's cost model: which lines carry the instructions)."""
    files: dict[int, str] = {}
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        m = re.match(r"\s*\.file\s+(\d+)\s+\"[^\"]*\"\s+\"([^\"]+)\"", l)
        if m:
            files[int(m.group(1))] = m.group(2)
        if start is None and re.match(r"^_Z\w*" + re.escape(fn) + r"\w*:", l):
            start = i
    per: dict[int, collections.Counter] = collections.defaultdict(collections.Counter)
    loc = None
    for l in lines[start + 1:]:
        s = l.strip()
        if s.startswith(".Lfunc_end"):
            break
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if m:
            f = files.get(int(m.group(1)), "")
            loc = int(m.group(2)) if f.endswith(src) else None
            continue
        if loc is None or not (lo <= loc <= hi) or not s or s[0] in ".;" or s.endswith(":"):
            continue
        op = s.split()[0]
        cat = ("lane" if op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")) else "valu" if op.startswith("v_")
               else "salu" if op.startswith("s_") else "ds" if op.startswith("ds_") else "vmem")
        per[loc][cat] += 1
    return {k: dict(v) for k, v in sorted(per.items())}
