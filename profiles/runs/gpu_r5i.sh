#!/bin/bash
# round 5: end-of-batch flushes vs immediate writes on the pipelined connections, interleaved x3
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5i
mkdir -p $out
for i in 1 2 3; do
  for v in default TT_DEFER_FLUSH=0; do
    env $( [ "$v" = default ] || echo $v ) timeout -k 10 300 python bench.py --steps 20 --warmup 5 --envelope-s 0 \
      --keda-messages 0 --direct-steps 0 --browser-steps 0 > $out/bench_${v//=/_}_$i.json 2> $out/bench_${v//=/_}_$i.err || exit $?
  done
done
