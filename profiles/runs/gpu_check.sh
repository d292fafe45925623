#!/usr/bin/env bash
# One GPU-box session: smoke, GPU tests, query-kernel bench + rocprofv3 profile, E2E bench (defaults).
# Every GPU step has its own time limit; steps are chained so the first failure stops the run.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd "$(dirname "$0")/../.."
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench_query.py --rows 100000000 --iters 20 --cpu > gpurun_out/bench_query.json 2> gpurun_out/bench_query.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o query -- python3 bench_query.py --rows 100000000 --iters 10 > gpurun_out/prof.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo ALL_OK
