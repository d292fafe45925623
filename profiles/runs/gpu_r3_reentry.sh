#!/usr/bin/env bash
# Round 3 re-entry check on a rebuilt tree: GPU tests, smoke(), one headline bench under the
# driver's flags.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3re_pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3re_smoke.log 2>&1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3re_bench.json 2> gpurun_out/r3re_bench.err
echo ALL_OK
