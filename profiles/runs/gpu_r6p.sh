#!/bin/bash
# round 6: markoverdue chunk sizes under the headline (headline only), then a rocprofv3 kernel
# trace of a headline run and its summary
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6p
mkdir -p $out
for c in 64 256; do
  timeout -k 10 240 python bench.py --steps 30 --warmup 5 --alt-steps 0 --envelope-s 0 --keda-messages 0 \
    --ingest-messages 0 --session-flows 0 --mark-chunk $c > $out/chunk$c.json 2> $out/chunk$c.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 20 --warmup 5 \
  --alt-steps 0 --envelope-s 0 --keda-messages 0 --ingest-messages 0 --session-flows 0 \
  > $out/prof_bench.json 2> $out/prof_bench.err || exit $?
db=$(find $out/prof -name '*.db' | head -1)
if [ -n "$db" ]; then python scripts/rocpd_summary.py "$db" "headline bench, round 6" > $out/kernels.md; fi
find $out/prof -name '*kernel_stats.csv' -exec cp {} $out/kernel_stats.csv \; 2>/dev/null
exit 0
