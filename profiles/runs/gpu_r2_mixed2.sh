#!/usr/bin/env bash
# Round 2: GPU tests (incl. the 1M-task sweep through the apps) and the mixed-load A/B after the
# native sweep lists.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/m2_pytest_gpu.log 2>&1
for i in 1 2 3; do
  for ms in 1000 0; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --overdue-sweep-ms $ms > gpurun_out/m2_${ms}_$i.json 2> gpurun_out/m2_${ms}_$i.err
  done
done
echo ALL_OK
