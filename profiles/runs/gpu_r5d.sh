#!/bin/bash
# round 5: the sweep with the front's query worker; markoverdue chunk 256 / 128 / 64
set -o pipefail
mkdir -p gpurun_out/r5d
for ch in 256 128 64; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --envelope-s 0 --direct-steps 0 --browser-steps 0 \
    --mark-chunk $ch > gpurun_out/r5d/bench_c$ch.json 2> gpurun_out/r5d/bench_c$ch.err || exit $?
done
