#!/bin/bash
# round 5: the sweep's markoverdue chunk (64 / 128 default / 256) on the current tree, headline
# only, 40 steps (about 9 sweeps per run), alternated twice
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5x
mkdir -p $out
for i in 1 2; do
  for c in 64 128 256; do
    timeout -k 10 300 python bench.py --steps 40 --warmup 5 --envelope-s 0 --keda-messages 0 --direct-steps 0 \
      --browser-steps 0 --mark-chunk $c > $out/bench_c${c}_$i.json 2> $out/bench_c${c}_$i.err || exit $?
  done
done
