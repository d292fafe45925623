#!/usr/bin/env bash
# Round 3 (c): GPU tests (page path now answers through pinned host mailboxes), the 1e8-row page
# benchmark + kernel trace, the sweep host-time profile on the GPU executor, the headline bench,
# and a 2-rank partitioned shared environment (both ranks on the box's one GPU).
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3c_pytest_gpu.log 2>&1
timeout -k 10 400 python bench_query.py --rows 100000000 --iters 20 --page --no-cpu-native > gpurun_out/r3c_bench_query.json 2> gpurun_out/r3c_bench_query.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3c_prof -o page -- python3 bench_query.py --rows 100000000 --iters 10 --page --no-cpu-native > gpurun_out/r3c_prof.log 2>&1
timeout -k 10 400 python scripts/sweep_sync_profile.py --gpu --profile > gpurun_out/r3c_sweep_gpu.json 2> gpurun_out/r3c_sweep_gpu.prof
timeout -k 10 400 python scripts/sweep_sync_profile.py > gpurun_out/r3c_sweep_cpu.json 2> gpurun_out/r3c_sweep_cpu.err
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3c_bench_fe.json 2> gpurun_out/r3c_bench_fe.err
HIP_VISIBLE_DEVICES=0 timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --shared-env > gpurun_out/r3c_shared2.json 2> gpurun_out/r3c_shared2.err
echo ALL_OK
