#!/usr/bin/env bash
# Round 3 (e): the overdue sweep after the background mirror sync and the short-page shortcut:
# GPU tests, the headline bench twice (sweep attribution in config.overdue_sweeps), the sweep
# profile on the GPU executor, and the 2-rank shared environment.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3e_pytest_gpu.log 2>&1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3e_fe_1.json 2> gpurun_out/r3e_fe_1.err
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3e_fe_2.json 2> gpurun_out/r3e_fe_2.err
timeout -k 10 400 python scripts/sweep_sync_profile.py --gpu > gpurun_out/r3e_sweep_gpu.json 2> gpurun_out/r3e_sweep_gpu.err
HIP_VISIBLE_DEVICES=0 timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29536 bench.py --gpus 2 --steps 10 --warmup 3 --shared-env > gpurun_out/r3e_shared2.json 2> gpurun_out/r3e_shared2.err
echo ALL_OK
