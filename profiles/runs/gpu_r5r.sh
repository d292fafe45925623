#!/bin/bash
# round 5: what the backing's append logs cost the headline -- logs on (default) vs
# TT_BACKING_LOGS=0, alternated x2; GPU tests first (the two new ones included)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5r
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gputests.log 2>&1 || exit $?
for i in 1 2; do
  for v in default TT_BACKING_LOGS=0; do
    env $( [ "$v" = default ] || echo $v ) timeout -k 10 300 python bench.py --steps 20 --warmup 5 --envelope-s 0 \
      --keda-messages 0 --direct-steps 0 --browser-steps 0 > $out/bench_${v//=/_}_$i.json 2> $out/bench_${v//=/_}_$i.err || exit $?
  done
done
