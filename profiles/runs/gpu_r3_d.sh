#!/usr/bin/env bash
# Round 3 (d): GPU tests; the headline bench (frontend entry, mTLS) alternated with mTLS off
# (two pairs) for profiles/r3_mtls_cost.md; 2 ranks env-per-rank next to the 2-rank shared
# environment of run (c); a kernel trace of the headline bench (the app-driven overdue sweep).
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3d_pytest_gpu.log 2>&1
for i in 1 2; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3d_fe_mtls_$i.json 2> gpurun_out/r3d_fe_mtls_$i.err
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 --mtls 0 > gpurun_out/r3d_fe_plain_$i.json 2> gpurun_out/r3d_fe_plain_$i.err
done
HIP_VISIBLE_DEVICES=0 timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/r3d_perrank2.json 2> gpurun_out/r3d_perrank2.err
HIP_VISIBLE_DEVICES=0 timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 --steps 10 --warmup 3 --shared-env > gpurun_out/r3d_shared2.json 2> gpurun_out/r3d_shared2.err
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d gpurun_out/r3d_prof_bench -o bench -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/r3d_prof_bench.json 2> gpurun_out/r3d_prof_bench.err
echo ALL_OK
