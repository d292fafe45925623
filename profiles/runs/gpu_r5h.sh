#!/bin/bash
# round 5: A/B of the batching knobs on the headline (no envelope): pipelined local connections
# with end-of-batch flushes (default), pipelined with immediate flushes, and neither
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5h
mkdir -p $out
for v in "default" "TT_DEFER_FLUSH=0" "TT_PIPELINE=0 TT_DEFER_FLUSH=0" "default"; do
  tag=$(echo "$v" | tr ' =' '__')
  env $( [ "$v" = default ] || echo $v ) timeout -k 10 300 python bench.py --steps 20 --warmup 5 --envelope-s 0 \
    --keda-messages 0 --direct-steps 0 > $out/bench_$tag.json 2> $out/bench_$tag.err || exit $?
  mv $out/bench_$tag.json $out/bench_${tag}_$(date +%s).json
done
