#!/usr/bin/env bash
# tt_scan_flat vs the program interpreter (tt_scan_eval): GPU numerics tests, the 1e8-row
# overdue-sweep A/B (bench_query.py reports both) and a kernel trace.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_columnar.py tests/test_backing.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/flat_pytest.log 2>&1
timeout -k 10 300 python bench_query.py --rows 100000000 --iters 20 > gpurun_out/flat_bench_query.json 2> gpurun_out/flat_bench_query.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_flat -o query -- python3 bench_query.py --rows 100000000 --iters 10 > gpurun_out/prof_flat.log 2>&1
echo ALL_OK
