#!/usr/bin/env bash
# Round 2: compaction that finds its own offsets from per-chunk counts (no full scan, no host
# sync mid-query, total to pinned memory) -- GPU tests, the 1e8-row query bench, kernel trace.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench_query.py --rows 100000000 --iters 30 --sorted --query > gpurun_out/bench_query.json 2> gpurun_out/bench_query.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_query4 -o query -- python3 bench_query.py --rows 100000000 --iters 10 > gpurun_out/prof_query4.log 2>&1
echo ALL_OK
