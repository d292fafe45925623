#!/bin/bash
# round 5: the headline with the new defaults, then A/Bs of the read path and the backing transport
set -o pipefail
mkdir -p gpurun_out/r5b
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r5b/bench.json 2> gpurun_out/r5b/bench.err || exit $?
TT_READ_PATH=bind timeout -k 10 300 python bench.py --steps 20 --warmup 5 --envelope-s 0 --direct-steps 0 \
  > gpurun_out/r5b/bench_bind.json 2> gpurun_out/r5b/bench_bind.err || exit $?
TT_BACKING_TRANSPORT=tcp timeout -k 10 300 python bench.py --steps 20 --warmup 5 --envelope-s 0 --direct-steps 0 \
  > gpurun_out/r5b/bench_tcp.json 2> gpurun_out/r5b/bench_tcp.err || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --envelope-s 0 --direct-steps 0 \
  > gpurun_out/r5b/bench_uds2.json 2> gpurun_out/r5b/bench_uds2.err
