#!/bin/bash
# round 6: run-to-run spread of the round-end tree, the driver's command x3 on one box
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6z
mkdir -p $out
for i in 1 2 3; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/bench$i.json 2> $out/bench$i.err || exit $?
done
exit 0
