#!/usr/bin/env bash
# Round 2: compaction with non-temporal id stores, A/B back to back (plus a kernel trace of each).
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_columnar.py -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/nt_pytest.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python bench_query.py --rows 100000000 --iters 30 --no-cpu-native > gpurun_out/nt_off_$i.json 2> gpurun_out/nt_off_$i.err
  timeout -k 10 200 python bench_query.py --rows 100000000 --iters 30 --no-cpu-native --compact-nt > gpurun_out/nt_on_$i.json 2> gpurun_out/nt_on_$i.err
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_nt" -o q -- python3 "$GRAFT_REPO_ROOT/bench_query.py" --rows 100000000 --iters 10 --no-cpu-native --compact-nt > "$GRAFT_REPO_ROOT/gpurun_out/prof_nt.log" 2>&1
echo ALL_OK
