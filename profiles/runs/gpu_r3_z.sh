#!/usr/bin/env bash
# Round 3 (z): headline bench (driver's flags) with traced sweeps and the store's hop stamps;
# then the same with 4 backing front threads (default 2).
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3z_bench.json 2> gpurun_out/r3z_bench.err
TT_BACKING_FRONT_THREADS=4 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3z_bench_ft4.json 2> gpurun_out/r3z_bench_ft4.err
echo ALL_OK
