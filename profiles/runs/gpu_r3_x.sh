#!/usr/bin/env bash
# Round 3 (x): top-k stamp test, then the headline bench (driver's flags) with traced sweeps.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_columnar.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3x_pytest.log 2>&1
tail -1 gpurun_out/r3x_pytest.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3x_bench.json 2> gpurun_out/r3x_bench.err
echo ALL_OK
