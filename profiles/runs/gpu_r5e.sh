#!/bin/bash
# round 5: GPU tests (scatter upload), then the sweep with one-launch uploads, chunk 128, bg sync 40 ms (x2) vs 100 ms
set -o pipefail
mkdir -p gpurun_out/r5e
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5e/gputests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --envelope-s 0 --direct-steps 0 --browser-steps 0 \
    > gpurun_out/r5e/bench_$i.json 2> gpurun_out/r5e/bench_$i.err || exit $?
done
TT_QUERY_MIRROR_SYNC_MS=100 timeout -k 10 240 python bench.py --steps 20 --warmup 5 --envelope-s 0 --direct-steps 0 \
  --browser-steps 0 > gpurun_out/r5e/bench_sync100.json 2> gpurun_out/r5e/bench_sync100.err
