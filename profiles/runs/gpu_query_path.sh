#!/usr/bin/env bash
# Whole paged state-query path on the GPU (select + ORDER BY + first page) at 1e7 and 1e8 rows,
# with a per-stage breakdown; GPU tests first.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd "$(dirname "$0")/../.."
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/qp_pytest.log 2>&1
timeout -k 10 300 python bench_query.py --rows 10000000 --iters 30 --query > gpurun_out/qp_1e7.json 2> gpurun_out/qp_1e7.err
timeout -k 10 300 python bench_query.py --rows 100000000 --iters 20 --query > gpurun_out/qp_1e8.json 2> gpurun_out/qp_1e8.err
timeout -k 10 600 python bench_query_e2e.py --docs 10000000 --accel gpu --queries 30 > gpurun_out/qp_e2e_10m.json 2> gpurun_out/qp_e2e_10m.err
echo ALL_OK
