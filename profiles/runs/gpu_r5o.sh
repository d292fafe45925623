#!/bin/bash
# round 5: one-pass task codec for the sweep pages: the page-plan probe, then two headline runs
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5o
mkdir -p $out
timeout -k 10 300 python profiles/runs/page_plan_probe.py > $out/plan.txt 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --envelope-s 0 --keda-messages 0 --direct-steps 0 \
    --browser-steps 0 > $out/bench_$i.json 2> $out/bench_$i.err || exit $?
done
