#!/usr/bin/env bash
# Round 2: createTask throughput with and without the concurrent app-driven overdue sweeps
# (GPU range queries every 1000 ms), alternating on one box (the driver's flags).
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for i in 1 2 3; do
  for ms in 1000 0; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --overdue-sweep-ms $ms > gpurun_out/mixed_${ms}_$i.json 2> gpurun_out/mixed_${ms}_$i.err
  done
done
echo ALL_OK
