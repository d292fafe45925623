#!/bin/bash
# round 6, final tree: rocprofv3 kernel trace of the driver's bench command and its summary
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6kern
mkdir -p $out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 20 --warmup 5 \
  > $out/bench.json 2> $out/bench.err || exit $?
db=$(find $out/prof -name '*.db' | head -1)
if [ -n "$db" ]; then python scripts/rocpd_summary.py "$db" "headline bench, round-6 final tree" > $out/kernels.md; fi
find $out/prof -name '*kernel_stats.csv' -exec cp {} $out/kernel_stats.csv \; 2>/dev/null
exit 0
