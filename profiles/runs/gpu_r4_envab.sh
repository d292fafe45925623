#!/usr/bin/env bash
# Round 4: A/B of one environment variable over the headline (driver's flags, no envelope),
# values alternated R4AB_REPS times; prints tasks/s, CPU per task, sweeps and the hottest threads.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
var=${R4AB_VAR:?}
out=gpurun_out/${R4AB_OUT:-r4ab}
mkdir -p $out
for i in $(seq 1 ${R4AB_REPS:-2}); do
  for v in ${R4AB_VALUES:?}; do
    env "$var=$v" timeout -k 10 400 python bench.py --steps 20 --warmup 5 --envelope-s 0 --direct-steps 0 > $out/bench_${v}_$i.json 2> $out/bench_${v}_$i.err
    python -c "
import json;d=json.load(open('$out/bench_${v}_$i.json'));c=d['config'];s=c['overdue_sweeps']
print('$var=$v', d['value'], c['cpu_us_per_task']['total'], s['sweep_p50_ms'], s['sweep_max_ms'], [r[1]+':'+str(r[2]) for r in c['hot_threads'][:5]])"
  done
done
echo ALL_OK
