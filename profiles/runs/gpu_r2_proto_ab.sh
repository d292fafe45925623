#!/usr/bin/env bash
# Round 2: sidecar API protocol A/B on one box (the driver's flags), back to back.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for i in 1 2; do
  for p in http grpc; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --api-protocol $p > gpurun_out/proto_${p}_$i.json 2> gpurun_out/proto_${p}_$i.err
  done
done
echo ALL_OK
