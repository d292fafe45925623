"""Merge the TT_PC_SAMPLE profiles (native/src/pcsample.hpp) of many processes by what they are
(``== dataplane <app id> pid N`` headers): per group, the share of each module and the busiest
symbols over all its processes.

    python scripts/pc_summary.py <dir or file prefix> [--top 25] [--json]
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import re
from collections import Counter, defaultdict


def parse(path: str):
    who, n = None, 0
    mods, syms = Counter(), Counter()
    part = None
    with open(path, errors="replace") as f:
        for ln in f:
            m = re.match(r"== (.*) pid \d+: (\d+) samples", ln)
            if m:
                who, n = m.group(1), int(m.group(2))
                continue
            if ln.startswith("-- by module"):
                part = "mod"
                continue
            if ln.startswith("-- by symbol"):
                part = "sym"
                continue
            m = re.match(r"\s*(\d+)\s+[\d.]+%\s+(\S+)(?:\s+(.*))?$", ln.rstrip("\n"))
            if not m:
                continue
            c = int(m.group(1))
            if part == "mod":
                mods[m.group(2)] += c
            elif part == "sym":
                syms[(m.group(2), (m.group(3) or "").strip())] += c
    return who, n, mods, syms


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("where")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    files = sorted(glob.glob(os.path.join(a.where, "*"))) if os.path.isdir(a.where) else sorted(glob.glob(a.where + ".*"))
    groups: dict[str, dict] = defaultdict(lambda: {"procs": 0, "samples": 0, "mods": Counter(), "syms": Counter()})
    for p in files:
        who, n, mods, syms = parse(p)
        if who is None:
            continue
        g = groups[who]
        g["procs"] += 1
        g["samples"] += n
        g["mods"].update(mods)
        g["syms"].update(syms)
    out = {}
    for who, g in sorted(groups.items()):
        n = g["samples"] or 1
        out[who] = {"processes": g["procs"], "samples": g["samples"],
                    "modules": {m: round(100 * c / n, 1) for m, c in g["mods"].most_common()},
                    "symbols": [[round(100 * c / n, 1), m, s] for (m, s), c in g["syms"].most_common(a.top)]}
    if a.json:
        print(json.dumps(out, indent=1))
        return
    for who, g in out.items():
        print(f"== {who}: {g['processes']} processes, {g['samples']} samples")
        print("   modules: " + ", ".join(f"{m} {v}%" for m, v in g["modules"].items()))
        for pct, m, s in g["symbols"]:
            print(f"   {pct:5.1f}%  {m:24s} {s}")


if __name__ == "__main__":
    main()
