#!/usr/bin/env bash
# Round 2: raw-code interpreter + 2-bit columns -- all GPU tests, smoke, the 1e8-row sweep with
# the fair CPU baseline, its kernel trace, and the state query through the stack (GPU).
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 400 python bench_query.py --rows 100000000 --iters 20 --sorted > gpurun_out/bq_final.json 2> gpurun_out/bq_final.err
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_scan2" -o q -- python3 "$GRAFT_REPO_ROOT/bench_query.py" --rows 100000000 --iters 10 --no-cpu-native > "$GRAFT_REPO_ROOT/gpurun_out/prof_scan2.log" 2>&1
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python bench_query_e2e.py --docs 10000000 --accel gpu --queries 20 > gpurun_out/qe2e_gpu.json 2> gpurun_out/qe2e_gpu.err
echo ALL_OK
