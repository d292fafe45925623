#!/usr/bin/env bash
# A/B of tt_scan_eval row groups per lane (1/2/4) + GPU tests.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd "$(dirname "$0")/../.."
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
for u in 1 2 4; do
  timeout -k 10 300 python bench_query.py --rows 100000000 --iters 30 --cpu --eval-groups $u > gpurun_out/bench_query_u$u.json 2> gpurun_out/bench_query_u$u.err
done
timeout -k 10 300 python bench_query.py --rows 100000000 --iters 20 --sorted > gpurun_out/bench_query.json 2> gpurun_out/bench_query.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o query -- python3 bench_query.py --rows 100000000 --iters 10 --sorted > gpurun_out/prof.log 2>&1
echo ALL_OK
