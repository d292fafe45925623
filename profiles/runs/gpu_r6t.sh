#!/bin/bash
# round 6: Python collection pauses (TT_GC_TRACE) lined up with the headline's steps
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6t
mkdir -p $out
TT_GC_TRACE=$out/gc timeout -k 10 300 python bench.py --steps 40 --warmup 5 --alt-steps 0 --envelope-s 0 \
  --keda-messages 0 --ingest-messages 0 --session-flows 0 > $out/bench.json 2> $out/bench.err || exit $?
python scripts/gc_steps.py $out/bench.err $out/gc > $out/gc_steps.txt
exit 0
