"""Line up the Python collection pauses of a bench run (``TT_GC_TRACE``, utils/gctrace.py) with
its timed steps: per step, its time and the pauses of 2 ms or more that started inside it.

    python scripts/gc_steps.py <bench stderr> <gc trace dir>
"""
from __future__ import annotations

import glob
import json
import os
import sys


def main(err: str, gcdir: str) -> None:
    diag = None
    for line in open(err):
        if line.startswith("{") and '"timed_wall_start"' in line:
            diag = json.loads(line)
    if diag is None:
        sys.exit("no diagnostics line with timed_wall_start")
    t0 = diag["timed_wall_start"]
    steps = [a for a, _ in diag["loadgen"]["steps_ms"]]
    pauses = []
    for f in glob.glob(os.path.join(gcdir, "gc-*.tsv")):
        who = os.path.basename(f)[3:-4]
        for row in open(f):
            w, gen, ms, _ = row.split("\t")
            pauses.append((float(w), who, int(gen), float(ms)))
    pauses.sort()
    edges, t = [], 0.0
    for ms in steps:
        edges.append((t, t + ms))
        t += ms
    med = sorted(steps)[len(steps) // 2]
    print(f"steps: {len(steps)}, median {med:.0f} ms; pauses >= 2 ms in the timed region:")
    for i, (a, b) in enumerate(edges):
        inside = [p for p in pauses if a <= (p[0] - t0) * 1e3 < b and p[3] >= 2.0]
        mark = " <" if steps[i] > 1.1 * med else ""
        desc = ", ".join(f"{who} g{gen} {ms:.1f}" for _, who, gen, ms in inside)
        print(f"  step {i + 1:2d}  {steps[i]:6.0f} ms{mark}  {desc}")
    by = {}
    for w, who, gen, ms in pauses:
        if 0 <= (w - t0) * 1e3 < t:
            k = (who.rsplit("-", 1)[0], gen)
            n, tot, mx = by.get(k, (0, 0.0, 0.0))
            by[k] = (n + 1, tot + ms, max(mx, ms))
    print("per process kind and generation (timed region): count, total ms, max ms")
    for (who, gen), (n, tot, mx) in sorted(by.items(), key=lambda kv: -kv[1][1]):
        print(f"  {who:48s} g{gen}  {n:4d}  {tot:8.1f}  {mx:6.1f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
