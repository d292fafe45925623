#!/usr/bin/env bash
# Round 2: glibc heap tuning A/B for every process of the stack (no trim / larger top pad, so
# request-sized allocations stop returning memory to the kernel and faulting it back in),
# alternating with the defaults on one box under the driver's flags.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/mal_off_$i.json 2> gpurun_out/mal_off_$i.err
  MALLOC_TRIM_THRESHOLD_=268435456 MALLOC_TOP_PAD_=67108864 MALLOC_MMAP_THRESHOLD_=67108864 \
    timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/mal_on_$i.json 2> gpurun_out/mal_on_$i.err
done
echo ALL_OK
