#!/bin/bash
# round 5: group commit of the backing's logs (default) vs one write per record
# (TT_BACKING_GROUP_COMMIT=0) vs no logs (TT_BACKING_LOGS=0), alternated x2
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5s
mkdir -p $out
for i in 1 2; do
  for v in default TT_BACKING_GROUP_COMMIT=0 TT_BACKING_LOGS=0; do
    env $( [ "$v" = default ] || echo $v ) timeout -k 10 300 python bench.py --steps 20 --warmup 5 --envelope-s 0 \
      --keda-messages 0 --direct-steps 0 --browser-steps 0 > $out/bench_${v//=/_}_$i.json 2> $out/bench_${v//=/_}_$i.err || exit $?
  done
done
