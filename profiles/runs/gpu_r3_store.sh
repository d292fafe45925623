#!/usr/bin/env bash
# Round 3 (re-entry): GPU tests, then the headline bench twice under the driver's flags after the
# store write-path / bulk encoding / API-log batching changes.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3s_pytest_gpu.log 2>&1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3s_bench_1.json 2> gpurun_out/r3s_bench_1.err
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3s_bench_2.json 2> gpurun_out/r3s_bench_2.err
echo ALL_OK
