#!/bin/bash
# round 5: wall vs thread CPU time of the page plan + program inside the headline (is the
# headline's extra over the 0.19 ms measured alone waiting or work?), headline only, 40 steps, x2
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5y
mkdir -p $out
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 5 --envelope-s 0 --keda-messages 0 --direct-steps 0 \
    --browser-steps 0 > $out/bench_$i.json 2> $out/bench_$i.err || exit $?
done
