#!/usr/bin/env bash
# Round 4: GPU tests (the repo's own radix pair sort replaces hipCUB), then the headline with the
# CPU duty cycle on the controller's Python tick vs on its native thread (dutycycle.hpp),
# alternated; the slowest sweep's spans and the per-app throttling of the timed region are in
# each bench line, and each run ends with the reference-envelope block.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
out=gpurun_out/r4sweep
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
tail -2 $out/pytest_gpu.log
for i in 1 2; do
  for duty in python native; do
    TT_CPU_DUTY=$duty timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $out/bench_${duty}_$i.json 2> $out/bench_${duty}_$i.err
    python -c "import json;d=json.load(open('$out/bench_${duty}_$i.json'));s=d['config']['overdue_sweeps'];print('$duty', d['value'], d['config']['cpu_us_per_task']['total'], s['sweep_p50_ms'], s['sweep_max_ms'], s['sweep_ms'])"
  done
done
echo ALL_OK
