#!/usr/bin/env bash
# Replica / concurrency sweep of the end-to-end bench (native app host), one box, back to back.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd "$(dirname "$0")/../.."
rm -f gpurun_out/sweep_*
for cfg in "6 3 288" "5 3 240" "7 3 336" "6 4 288" "5 2 240" "6 3 384" "6 3 288"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 40 --warmup 5 --api-replicas $1 --processor-replicas $2 --concurrency $3 > gpurun_out/sweep_$1_$2_$3.json 2> gpurun_out/sweep_$1_$2_$3.err || true
done
echo ALL_OK
