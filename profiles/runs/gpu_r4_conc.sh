#!/usr/bin/env bash
# Round 4: with the native routes the per-replica caps no longer bind (0 % stopped): sweep the
# load generator's in-flight window (default 48 per frontend replica = 192) on one box.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
out=gpurun_out/${R4CONC_OUT:-r4conc}
mkdir -p $out
for i in 1 2; do
  for conc in ${R4CONC_LIST:-192 288 384}; do
    timeout -k 10 400 python bench.py --steps 20 --warmup 5 --envelope-s 0 --direct-steps 0 --concurrency $conc ${R4CONC_EXTRA:-} > $out/bench_${conc}_$i.json 2> $out/bench_${conc}_$i.err
    python -c "import json;d=json.load(open('$out/bench_${conc}_$i.json'));c=d['config'];u=c['cpu_us_per_task'];t=c['cpu_limits']['throttling_in_timed_region'];print('conc=$conc', d['value'], u['total'], c['create_latency_p50_ms'], c['create_latency_p99_ms'], c['overdue_sweeps']['sweep_p50_ms'], {k: v['stopped_share'] for k, v in t.items()})"
  done
done
echo ALL_OK
