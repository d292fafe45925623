#!/usr/bin/env bash
# Round 3 final check: GPU tests, smoke(), the headline bench under the driver's flags (twice),
# a kernel trace of the headline (app-driven sweep), and the 2-rank partitioned environment.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3final2_pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3final2_smoke.log 2>&1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3final2_bench_1.json 2> gpurun_out/r3final2_bench_1.err
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3final2_bench_2.json 2> gpurun_out/r3final2_bench_2.err
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d gpurun_out/r3final2_prof_bench -o bench -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/r3final2_prof_bench.json 2> gpurun_out/r3final2_prof_bench.err
HIP_VISIBLE_DEVICES=0 timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 10 --warmup 3 --shared-env > gpurun_out/r3final2_shared2.json 2> gpurun_out/r3final2_shared2.err
echo ALL_OK
