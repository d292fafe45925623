#!/usr/bin/env bash
# Round 3 (k): the radix-select top-k -- GPU tests, then the 1e8-row page benchmark + kernel trace.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3k_pytest_gpu.log 2>&1
timeout -k 10 400 python bench_query.py --rows 100000000 --iters 20 --page --no-cpu-native > gpurun_out/r3k_bench_query.json 2> gpurun_out/r3k_bench_query.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3k_prof -o page -- python3 bench_query.py --rows 100000000 --iters 10 --page --no-cpu-native > gpurun_out/r3k_prof.log 2>&1
echo ALL_OK
