#!/usr/bin/env bash
# Round 3 (m): placement A/B -- the stack on the GPU's NUMA node (every hardware thread) vs
# one hardware thread per physical core of that node -- alternated twice on one box.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for i in 1 2; do
  TT_BENCH_PIN=node timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3m_node_$i.json 2> gpurun_out/r3m_node_$i.err
  TT_BENCH_PIN=phys timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3m_phys_$i.json 2> gpurun_out/r3m_phys_$i.err
done
echo ALL_OK
