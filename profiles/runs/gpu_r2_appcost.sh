#!/usr/bin/env bash
# Round 2: service CPU per task after the native codec / glue work -- smoke, GPU tests, the
# headline bench under the driver's flags, and the per-process attribution tools on the box.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err
timeout -k 10 300 python scripts/app_cost.py > gpurun_out/app_cost.log 2>&1
timeout -k 10 300 python scripts/host_cost.py --service api > gpurun_out/host_cost_api.log 2>&1
timeout -k 10 300 python scripts/host_cost.py --service processor > gpurun_out/host_cost_proc.log 2>&1
echo ALL_OK
