#!/usr/bin/env bash
# Round 4: the repo's own LSD radix pair sort (hip/radix_pairs.hip, replacing hipCUB): its GPU
# tests, then the 1e8-row ORDER BY taskDueDate DESC (31.5 M selected rows) timings and a kernel
# trace.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
out=gpurun_out/${R4RADIX_OUT:-r4radix}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_columnar.py -x -q -m gpu -k "radix or ordered or page or sort" --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
tail -2 $out/pytest.log
timeout -k 10 300 python bench_query.py --rows 100000000 --iters 20 --sorted > $out/bench.json 2> $out/bench.err
cat $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o q -- python3 bench_query.py --rows 100000000 --iters 5 --sorted > $out/prof.log 2>&1
echo ALL_OK
