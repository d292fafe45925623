#!/usr/bin/env bash
# Prefetching evaluator (tt_scan_eval_pf) vs the interpreter (tt_scan_eval_t<2>): GPU numerics
# tests, then bench_query A/B (alternating), then a kernel trace of both.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd "$(dirname "$0")/.."
rm -rf gpurun_out/pf_*
timeout -k 10 300 python -u -m pytest tests/test_columnar.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pf_pytest.log 2>&1
for i in 1 2; do
  for cfg in "interp 0" "pf 2" "pf 1"; do
    set -- $cfg
    timeout -k 10 300 python bench_query.py --rows 100000000 --iters 30 --eval-kernel $1 --pf-groups $2 > gpurun_out/pf_$1_$2_$i.json 2> gpurun_out/pf_$1_$2_$i.err
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pf_prof -o pf -- python3 bench_query.py --rows 100000000 --iters 10 --eval-kernel pf > gpurun_out/pf_prof.log 2>&1
echo ALL_OK
