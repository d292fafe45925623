#!/usr/bin/env bash
# Round 2: scan sensitivity to loads in flight (row groups per lane) with 2-bit columns.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_columnar.py -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu_col.log 2>&1
for u in 1 2 4 8; do
  timeout -k 10 200 python bench_query.py --rows 100000000 --iters 20 --eval-groups $u --no-cpu-native > gpurun_out/bq_u$u.json 2> gpurun_out/bq_u$u.err
done
echo ALL_OK
