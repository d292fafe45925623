#!/usr/bin/env bash
# The driver's multi-rank bench launch, rehearsed with 2 ranks on one box (each rank runs its own
# environment sized to half the box's CPU share).
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd "$(dirname "$0")/../.."
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/bench_2rank.json 2> gpurun_out/bench_2rank.err
echo ALL_OK
