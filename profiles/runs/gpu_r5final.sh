#!/bin/bash
# round 5, final tree: GPU tests, smoke(), the driver's bench command twice, then a rocprofv3
# kernel trace of a headline-only run
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5final
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gputests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/bench_$i.json 2> $out/bench_$i.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 20 --warmup 5 \
  --envelope-s 0 --keda-messages 0 --direct-steps 0 --browser-steps 0 > $out/prof_bench.json 2> $out/prof_bench.err
