#!/usr/bin/env bash
# GPU numerics for the query kernels + the rank-encode kernel time (rocprofv3 kernel trace).
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_columnar.py tests/test_backing.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/re_pytest.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_re -o query -- python3 bench_query.py --rows 100000000 --iters 10 > gpurun_out/prof_re.log 2>&1
echo ALL_OK
