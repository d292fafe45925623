#!/usr/bin/env bash
# Round 3 (aa): headline bench (driver's flags), traced sweeps with the query's return-path stamps.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3aa_bench.json 2> gpurun_out/r3aa_bench.err
echo ALL_OK
