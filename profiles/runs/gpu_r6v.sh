#!/bin/bash
# round 6: the driver's command x2 with the staggered store shards and one load generator process
# for the warmup and the timed steps
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6v
mkdir -p $out
for i in 1 2; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench$i.json 2> $out/bench$i.err || exit $?
done
exit 0
