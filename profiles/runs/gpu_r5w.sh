#!/bin/bash
# round 5: the driver's command twice after the allocation cuts in the HTTP layer (headers moved,
# answers written in place, shared TLS peer names, run-based JSON escaping), then the data
# planes' PC samples of a headline-only run
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5w
mkdir -p $out/pcs
for i in 1 2; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/bench_$i.json 2> $out/bench_$i.err || exit $?
done
TT_PC_SAMPLE=$PWD/$out/pcs/prof timeout -k 10 300 python bench.py --steps 20 --warmup 5 --envelope-s 0 \
  --direct-steps 0 --browser-steps 0 > $out/pcs_bench.json 2> $out/pcs_bench.err
