#!/usr/bin/env bash
# Round 3 (h): headline bench twice with the sweep's in-situ breakdown (timed region only,
# sweeper running from the warmup on), after the GPU tests.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3h_pytest_gpu.log 2>&1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3h_fe_1.json 2> gpurun_out/r3h_fe_1.err
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3h_fe_2.json 2> gpurun_out/r3h_fe_2.err
echo ALL_OK
