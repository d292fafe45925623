#!/usr/bin/env bash
# Round 2 re-entry check: smoke, GPU tests, headline bench under the driver's flags and the
# defaults, and a kernel-trace profile of the headline bench (GPU work of the concurrent sweeps).
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench -- python3 bench.py --steps 10 --warmup 2 > gpurun_out/prof_bench.log 2>&1
echo ALL_OK
