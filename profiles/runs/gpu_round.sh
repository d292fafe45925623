#!/usr/bin/env bash
# GPU tests, query kernels (fused select A/B + ordering) with profile, end-to-end state query at 10M docs.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd "$(dirname "$0")/../.."
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench_query.py --rows 100000000 --iters 20 --sorted > gpurun_out/bench_query.json 2> gpurun_out/bench_query.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o query -- python3 bench_query.py --rows 100000000 --iters 10 --sorted > gpurun_out/prof.log 2>&1
timeout -k 10 600 python bench_query_e2e.py --docs 10000000 --accel gpu --queries 20 > gpurun_out/qe2e_gpu_10m.json 2> gpurun_out/qe2e_gpu_10m.err
echo ALL_OK
