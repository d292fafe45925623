#!/usr/bin/env bash
# Round 3 (j): GPU tests (incl. the top-k at every candidate count),
# the 1e8-row page benchmark + kernel trace, then the headline bench twice (sweep breakdown).
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3j_pytest_gpu.log 2>&1
timeout -k 10 400 python bench_query.py --rows 100000000 --iters 20 --page --no-cpu-native > gpurun_out/r3j_bench_query.json 2> gpurun_out/r3j_bench_query.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3j_prof -o page -- python3 bench_query.py --rows 100000000 --iters 10 --page --no-cpu-native > gpurun_out/r3j_prof.log 2>&1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3j_fe_1.json 2> gpurun_out/r3j_fe_1.err
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3j_fe_2.json 2> gpurun_out/r3j_fe_2.err
echo ALL_OK
