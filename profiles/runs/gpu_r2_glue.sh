#!/usr/bin/env bash
# Round 2: device-side tile offsets (no mid-query host sync) -- GPU tests, the 1e8-row query
# bench + its kernel trace, and the headline bench over the native gRPC transport.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench_query.py --rows 100000000 --iters 20 --sorted --query > gpurun_out/bench_query.json 2> gpurun_out/bench_query.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_query -o query -- python3 bench_query.py --rows 100000000 --iters 10 > gpurun_out/prof_query.log 2>&1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_http.json 2> gpurun_out/bench_http.err
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --api-protocol grpc > gpurun_out/bench_grpc.json 2> gpurun_out/bench_grpc.err
echo ALL_OK
