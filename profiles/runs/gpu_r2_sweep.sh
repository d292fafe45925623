#!/usr/bin/env bash
# Round 2: GPU tests (incl. the 1M-task app-driven overdue sweep), the sweep bench + its
# rocprofv3 kernel trace, and the headline bench with / without concurrent sweeps.
# Every GPU step has its own time limit; steps are chained so the first failure stops the run.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench_overdue.py --tasks 1000000 --accel gpu > gpurun_out/overdue_gpu.json 2> gpurun_out/overdue_gpu.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_overdue -o sweep -- python3 bench_overdue.py --tasks 1000000 --accel gpu > gpurun_out/prof_overdue.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 400 python bench.py --overdue-sweep-ms 0 > gpurun_out/bench_nosweep.json 2> gpurun_out/bench_nosweep.err
echo ALL_OK
