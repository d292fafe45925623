#!/usr/bin/env python3
"""Sort-only probe of ``tt_sort_pairs`` (ops/hip/radix_pairs.hip) for kernel traces and counter
passes: ``--n`` random (key, row) pairs with keys below 2**``--bits`` shaped like the query path's
packed keys (a few distinct high digits over a random low part), timed over ``--iters`` sorts and
checked against ``torch.sort(stable=True)``.  One JSON line."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=31_498_523)
    ap.add_argument("--bits", type=int, default=36)
    ap.add_argument("--high-values", type=int, default=336, help="distinct values of the bits above 27")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()

    import torch

    from aca_dotnet_workshop_amd.ops.gpu import GpuKernels

    k = GpuKernels("cuda:0")
    dev = k.device
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    low_bits = min(27, a.bits)
    low = torch.randint(0, 1 << low_bits, (a.n,), device=dev, generator=g, dtype=torch.int64)
    high = torch.zeros_like(low)
    if a.bits > low_bits:
        vals = min(a.high_values, 1 << (a.bits - low_bits))
        high = torch.randint(0, vals, (a.n,), device=dev, generator=g, dtype=torch.int64) << low_bits
    keys = high | low
    rows = torch.randperm(a.n, device=dev, generator=g, dtype=torch.int32)
    for _ in range(a.warmup):
        out = k._sorted_rows(keys, rows, a.bits)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        out = k._sorted_rows(keys, rows, a.bits)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    k.check_sort()
    _, idx = torch.sort(keys, stable=True)
    match = bool(torch.equal(out, rows[idx]))
    print(json.dumps({"n": a.n, "bits": a.bits, "passes": (a.bits + 7) // 8, "sort_ms": round(dt * 1e3, 4),
                      "pairs_per_s": round(a.n / dt, 1), "match": match}), flush=True)


if __name__ == "__main__":
    main()
