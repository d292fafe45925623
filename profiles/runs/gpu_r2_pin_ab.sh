#!/usr/bin/env bash
# Per-rank CPU pinning A/B: the driver's multi-rank launch rehearsed with 2 ranks on one box,
# pinned (default) vs TT_BENCH_PIN=0, twice each, plus the host's NUMA/CPU layout.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
{ nproc; python -c "import os; print(len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max || true
  for n in /sys/devices/system/node/node*/cpulist; do echo "$n $(cat $n)"; done; } > gpurun_out/pin_host.txt 2>&1
port=29540
for i in 1 2; do
  for mode in 1 0; do
    port=$((port + 1))
    TT_BENCH_PIN=$mode timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --steps 20 --warmup 5 \
      > gpurun_out/pin_ab_${mode}_$i.json 2> gpurun_out/pin_ab_${mode}_$i.err
  done
done
echo ALL_OK
