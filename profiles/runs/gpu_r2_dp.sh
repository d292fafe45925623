#!/usr/bin/env bash
# Round 2: headline bench after the data-plane JSON / tracer work, with the kernel-mode share of
# every process role (bench.py's cpu_cores_busy_kernel_mode), three runs under the driver's flags.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/dp_$i.json 2> gpurun_out/dp_$i.err
done
echo ALL_OK
