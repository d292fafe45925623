#!/usr/bin/env bash
# Round 4: the busiest single threads of the headline's timed region (config.hot_threads).
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
out=gpurun_out/${R4HOT_OUT:-r4hot}
mkdir -p $out
for i in ${R4HOT_RUNS:-1 2}; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --envelope-s 0 --direct-steps 0 ${R4HOT_ARGS:-} > $out/bench_$i.json 2> $out/bench_$i.err
  python -c "
import json;d=json.load(open('$out/bench_$i.json'));c=d['config'];s=c['overdue_sweeps']
print('run $i', d['value'], c['cpu_us_per_task']['total'], s['sweep_p50_ms'], s['sweep_max_ms'])
for r in c['hot_threads']: print('   ', r)"
done
echo ALL_OK
