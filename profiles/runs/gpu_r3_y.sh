#!/usr/bin/env bash
# Round 3 (y): top-k stamp test, then the headline bench (driver's flags) with traced sweeps.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3y_bench.json 2> gpurun_out/r3y_bench.err
echo ALL_OK
