#!/usr/bin/env bash
# Backing-front shard threads (TT_BACKING_FRONT_THREADS) A/B for the 1-rank bench, alternating.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd "$(dirname "$0")/../.."
rm -f gpurun_out/bt_*
for i in 1 2; do
  for t in 2 4; do
    TT_BACKING_FRONT_THREADS=$t timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/bt_${t}_$i.json 2> gpurun_out/bt_${t}_$i.err
  done
done
echo ALL_OK
