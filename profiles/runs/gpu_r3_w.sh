#!/usr/bin/env bash
# Round 3 (w): register sort + merge tree top-k -- GPU tests, 1e8-row page benchmark + kernel trace.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3w_pytest_gpu.log 2>&1
tail -2 gpurun_out/r3w_pytest_gpu.log
timeout -k 10 400 python bench_query.py --rows 100000000 --iters 20 --page --no-cpu-native > gpurun_out/r3w_bench_query.json 2> gpurun_out/r3w_bench_query.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3w_prof -o page -- python3 bench_query.py --rows 100000000 --iters 10 --page --no-cpu-native > gpurun_out/r3w_prof.log 2>&1
echo ALL_OK
