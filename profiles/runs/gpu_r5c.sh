#!/bin/bash
# round 5: headline with native read path + query front + batched log lines; A/B read path
set -o pipefail
mkdir -p gpurun_out/r5c
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --envelope-s 0 --keda-messages 0 --direct-steps 0 \
  > gpurun_out/r5c/bench.json 2> gpurun_out/r5c/bench.err || exit $?
TT_READ_PATH=bind timeout -k 10 300 python bench.py --steps 20 --warmup 5 --envelope-s 0 --direct-steps 0 \
  > gpurun_out/r5c/bench_bind.json 2> gpurun_out/r5c/bench_bind.err || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --envelope-s 0 --keda-messages 0 --direct-steps 0 \
  > gpurun_out/r5c/bench2.json 2> gpurun_out/r5c/bench2.err
