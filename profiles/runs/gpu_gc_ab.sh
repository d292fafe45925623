#!/usr/bin/env bash
# Server GC tuning A/B (TT_GC_GEN0=0: interpreter defaults; 20000: tuned), alternating runs.
set -euo pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for i in 1 2 3; do
  for g in 0 20000; do
    TT_GC_GEN0=$g timeout -k 10 300 python bench.py > gpurun_out/gc_${g}_$i.json 2> gpurun_out/gc_${g}_$i.err
  done
done
echo ALL_OK
