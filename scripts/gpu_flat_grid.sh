#!/usr/bin/env bash
# tt_scan_flat grid sweep (grid-stride workgroups vs one per tile), 1e8-row overdue sweep.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_columnar.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/flat_pytest.log 2>&1
for g in 0 1024 2048 4096; do
  timeout -k 10 200 python bench_query.py --rows 100000000 --iters 30 --flat-grid $g > gpurun_out/flat_grid_$g.json 2> gpurun_out/flat_grid_$g.err
done
echo ALL_OK
