#!/usr/bin/env bash
# Round 2: 6+3 vs 7+3 replicas (the driver's flags), alternating on one box.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for i in 1 2 3; do
  for t in "6 3" "7 3"; do
    set -- $t
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --api-replicas $1 --processor-replicas $2 \
      > gpurun_out/tab_$1_$2_$i.json 2> gpurun_out/tab_$1_$2_$i.err
  done
done
echo ALL_OK
