#!/usr/bin/env bash
# Round 3 (q): full selections sized from the previous count (no clone): GPU tests, then the
# 1e8-row scan benchmark (filter + compaction) and its kernel trace.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3q_pytest_gpu.log 2>&1
timeout -k 10 400 python bench_query.py --rows 100000000 --iters 20 --page --no-cpu-native > gpurun_out/r3q_bench_query.json 2> gpurun_out/r3q_bench_query.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3q_prof -o scan -- python3 bench_query.py --rows 100000000 --iters 10 --no-cpu-native > gpurun_out/r3q_prof.log 2>&1
echo ALL_OK
