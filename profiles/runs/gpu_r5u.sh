#!/bin/bash
# round 5: the load generator's concurrency -- 192 (the default, 48 per frontend replica) vs 256
# vs 320 in flight, alternated x2 (headline only): is the environment latency- or CPU-bound?
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5u
mkdir -p $out
for i in 1 2; do
  for c in 192 256 320; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --envelope-s 0 --keda-messages 0 --direct-steps 0 \
      --browser-steps 0 --concurrency $c > $out/bench_c${c}_$i.json 2> $out/bench_c${c}_$i.err || exit $?
  done
done
