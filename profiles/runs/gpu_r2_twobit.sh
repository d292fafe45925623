#!/usr/bin/env bash
# Round 2: 2-bit boolean columns -- GPU tests, the 1e8-row sweep (GPU vs fair CPU baseline), a
# kernel trace of it, and the state query through the stack on the CPU path (top-k pages).
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 400 python bench_query.py --rows 100000000 --iters 20 > gpurun_out/bq_2bit.json 2> gpurun_out/bq_2bit.err
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_2bit" -o q -- python3 "$GRAFT_REPO_ROOT/bench_query.py" --rows 100000000 --iters 10 --no-cpu-native > "$GRAFT_REPO_ROOT/gpurun_out/prof_2bit.log" 2>&1
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python bench_query_e2e.py --docs 10000000 --accel cpu --queries 20 > gpurun_out/qe2e_cpu.json 2> gpurun_out/qe2e_cpu.err
echo ALL_OK
