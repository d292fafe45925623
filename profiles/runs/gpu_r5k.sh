#!/bin/bash
# round 5: native string ranks (strrank.hpp) in the sweep's sort plan; mirror background sync
# every 40 ms (default) vs 20 ms, interleaved x2; GPU tests first
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5k
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gputests.log 2>&1 || exit $?
for i in 1 2; do
  for v in default TT_QUERY_MIRROR_SYNC_MS=20; do
    env $( [ "$v" = default ] || echo $v ) timeout -k 10 300 python bench.py --steps 20 --warmup 5 --envelope-s 0 \
      --keda-messages 0 --direct-steps 0 --browser-steps 0 > $out/bench_${v//=/_}_$i.json 2> $out/bench_${v//=/_}_$i.err || exit $?
  done
done
