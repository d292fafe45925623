#!/usr/bin/env bash
# Round 3 (p): the split page gather (GPU tests, 1e8-row page bench + kernel trace), then the
# headline's replica / concurrency sweep (one thread per core, the default placement).
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3p_pytest_gpu.log 2>&1
timeout -k 10 400 python bench_query.py --rows 100000000 --iters 20 --page --no-cpu-native > gpurun_out/r3p_bench_query.json 2> gpurun_out/r3p_bench_query.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3p_prof -o page -- python3 bench_query.py --rows 100000000 --iters 10 --page --no-cpu-native > gpurun_out/r3p_prof.log 2>&1
run() { local tag=$1; shift; timeout -k 10 600 python bench.py --steps 20 --warmup 5 --direct-steps 0 "$@" > gpurun_out/r3p_$tag.json 2> gpurun_out/r3p_$tag.err; }
run base
run fe4_api5 --api-replicas 5
run fe3_api4 --frontend-replicas 3
run fe5_api5 --frontend-replicas 5 --api-replicas 5
run c256 --concurrency 256
run c128 --concurrency 128
run proc3 --processor-replicas 3
echo ALL_OK
