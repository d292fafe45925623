#!/usr/bin/env bash
# Round 2: replica sizing after the service-cost cuts (the driver's flags, one box, back to back).
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for t in "6 3" "7 2" "7 3" "8 2" "6 2"; do
  set -- $t
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --api-replicas $1 --processor-replicas $2 \
    > gpurun_out/topo_$1_$2.json 2> gpurun_out/topo_$1_$2.err
done
echo ALL_OK
