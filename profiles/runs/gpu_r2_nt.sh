#!/usr/bin/env bash
# Round 2: non-temporal loads / stores in the scan pipeline, A/B back to back.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_columnar.py -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/nt_pytest.log 2>&1
for i in 1 2; do
  for v in "0 0" "1 0" "1 1" "0 1"; do
    set -- $v
    timeout -k 10 200 python bench_query.py --rows 100000000 --iters 30 --no-cpu-native --compact-nt $1 --eval-nt $2 \
      > gpurun_out/nt_c$1_e$2_$i.json 2> gpurun_out/nt_c$1_e$2_$i.err
  done
done
echo ALL_OK
