#!/bin/bash
# round 6: the headline's per-step times with the store's shards growing at staggered points,
# 40 steps (store 82k -> 737k documents), then a second 20-step run
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6u
mkdir -p $out
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --alt-steps 0 --envelope-s 0 \
  --keda-messages 0 --ingest-messages 0 --session-flows 0 > $out/bench40.json 2> $out/bench40.err || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --alt-steps 0 --envelope-s 0 \
  --keda-messages 0 --ingest-messages 0 --session-flows 0 > $out/bench20.json 2> $out/bench20.err || exit $?
exit 0
