#!/bin/bash
# round 6: where the external-ingest block's time goes (its hot threads, stderr line)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r6ing}
mkdir -p $out
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --alt-steps 0 --envelope-s 0 --keda-messages 0 \
  --session-flows 0 --browser-steps 0 --direct-steps 0 --ingest-messages 8192 > $out/bench.json 2> $out/bench.err || exit $?
exit 0
