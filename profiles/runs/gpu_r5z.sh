#!/bin/bash
# round 5: where the page plan's CPU goes inside the headline (ranks / tails / upload / rebuilds),
# after the columnar GPU tests
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5z
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_columnar.py tests/test_gpu_overdue_sweep.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/gputests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 5 --envelope-s 0 --keda-messages 0 --direct-steps 0 \
    --browser-steps 0 > $out/bench_$i.json 2> $out/bench_$i.err || exit $?
done
