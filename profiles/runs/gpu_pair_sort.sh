#!/usr/bin/env bash
# Pair radix sort over the used key bits vs torch.sort argsort + gather: GPU numerics + A/B +
# kernel trace of the sorted overdue sweep.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_columnar.py tests/test_backing.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/ps_pytest.log 2>&1
timeout -k 10 300 python bench_query.py --rows 100000000 --iters 20 --sorted > gpurun_out/ps_bench.json 2> gpurun_out/ps_bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ps -o q -- python3 bench_query.py --rows 100000000 --iters 5 --sorted > gpurun_out/prof_ps.log 2>&1
echo ALL_OK
