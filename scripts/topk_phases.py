"""Per-phase shader-clock breakdown of ``tt_page_topk`` (ops/hip/page_topk.hip).

Runs the kernel alone over synthetic candidates (the shape of the 1e8-row overdue page: a few
thousand clustered keys, k = 1,000) with its ``stamps`` argument set, and prints one JSON line
per candidate count: the clock deltas of load+min/max, the radix select, the compaction, the
LDS sort and the write-out (clock64 ticks; the last field converts with the device clock).

    python scripts/topk_phases.py [--out gpurun_out/topk_phases.json]
"""
from __future__ import annotations

import argparse
import json
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--k", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    import torch
    from aca_dotnet_workshop_amd.ops.gpu import GpuKernels
    kern = GpuKernels()
    dev = kern.device
    names = ["load_minmax", "radix_select", "compact", "sort", "write"]
    rows_out = []
    for n in (700, 1000, 1500, 2600, 4096, 8192):
        rng = np.random.default_rng(n)
        keys = (rng.integers(0, 1 << 40, n, dtype=np.int64) << 20) | np.arange(n, dtype=np.int64)
        rows = rng.permutation(n).astype(np.int32)
        dk, dr = torch.from_numpy(keys).to(dev), torch.from_numpy(rows).to(dev)
        stamps = torch.zeros(6, dtype=torch.int64, device=dev)
        acc = np.zeros(5)
        seen = np.zeros(5)
        order = rows[np.argsort(keys.astype(np.uint64), kind="stable")]
        for r in range(a.reps + 5):
            stamps.zero_()
            got, info = kern.page_topk(dk, dr, a.k, 0, np.iinfo(np.uint64).max, stamps=stamps)
            s = stamps.cpu().numpy()
            if r >= 5:  # a phase the branch skipped (n <= k: no select) leaves its stamp at 0
                idx = [i for i in range(6) if s[i] != 0]
                for lo, hi in zip(idx, idx[1:]):
                    acc[hi - 1] += s[hi] - s[lo]
                    seen[hi - 1] += 1
        assert got.tolist() == order[:min(n, a.k)].tolist()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            kern.page_topk(dk, dr, a.k, 0, np.iinfo(np.uint64).max)
        wall_us = (time.perf_counter() - t0) / a.reps * 1e6
        ph = {nm: round(float(v / c), 1) for nm, v, c in zip(names, acc, seen) if c}
        rec = {"n": n, "k": a.k, "ticks": ph, "total_ticks": round(float(acc.sum() / a.reps), 1),
               "call_wall_us": round(wall_us, 1)}
        rows_out.append(rec)
        print(json.dumps(rec), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows_out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
