#!/usr/bin/env bash
# Round 2 end-of-session check: smoke, every GPU test, the headline bench under the driver's
# flags and with its defaults, the gRPC transport, and a kernel trace of the headline bench.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 180 --timeout-method thread > gpurun_out/final_pytest_gpu.log 2>&1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/final_bench_driver.json 2> gpurun_out/final_bench_driver.err
timeout -k 10 400 python bench.py > gpurun_out/final_bench_default.json 2> gpurun_out/final_bench_default.err
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --api-protocol grpc > gpurun_out/final_bench_grpc.json 2> gpurun_out/final_bench_grpc.err
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/final_prof_bench" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/final_prof_bench.log" 2>&1
echo ALL_OK
