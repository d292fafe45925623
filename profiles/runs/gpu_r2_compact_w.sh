#!/usr/bin/env bash
# Round 2: wave-independent compaction (tile offsets in one block) vs the per-block offset search,
# back to back on one box, plus a kernel trace of each.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_columnar.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/cw_pytest.log 2>&1
for i in 1 2; do
  for m in 1 0; do
    timeout -k 10 200 python bench_query.py --rows 100000000 --iters 30 --no-cpu-native --compact-mode $m > gpurun_out/cw_m${m}_$i.json 2> gpurun_out/cw_m${m}_$i.err
  done
done
cd /tmp
for m in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_cw$m" -o q -- python3 "$GRAFT_REPO_ROOT/bench_query.py" --rows 100000000 --iters 10 --no-cpu-native --compact-mode $m > "$GRAFT_REPO_ROOT/gpurun_out/prof_cw$m.log" 2>&1
done
echo ALL_OK
