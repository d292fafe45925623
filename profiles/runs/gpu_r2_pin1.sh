#!/usr/bin/env bash
# Single-rank CPU placement A/B under the driver's flags: unpinned vs first NUMA node vs the
# first 32 / 16 CPUs of that node (whole cores), alternated twice.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for i in 1 2; do
  for mode in 0 node 32 16; do
    TT_BENCH_PIN=$mode timeout -k 10 240 python bench.py --steps 20 --warmup 5 \
      > gpurun_out/pin1_${mode}_$i.json 2> gpurun_out/pin1_${mode}_$i.err
  done
done
echo ALL_OK
