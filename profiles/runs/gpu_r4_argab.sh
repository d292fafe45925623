#!/usr/bin/env bash
# Round 4: A/B of bench.py argument sets over the headline (driver's flags, no envelope),
# alternated R4ARG_REPS times. R4ARG_SETS: sets separated by ';' (an empty set = the defaults).
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
out=gpurun_out/${R4ARG_OUT:-r4arg}
mkdir -p $out
IFS=';' read -ra sets <<< "${R4ARG_SETS:?}"
for i in $(seq 1 ${R4ARG_REPS:-2}); do
  k=0
  for s in "${sets[@]}"; do
    k=$((k+1))
    timeout -k 10 400 python bench.py --steps 20 --warmup 5 --envelope-s 0 --direct-steps 0 $s > $out/bench_${k}_$i.json 2> $out/bench_${k}_$i.err
    python -c "
import json;d=json.load(open('$out/bench_${k}_$i.json'));c=d['config'];s=c['overdue_sweeps']
print('[$s]', d['value'], c['cpu_us_per_task']['total'], s['sweep_p50_ms'], s['sweep_max_ms'], [r[1]+':'+str(r[2]) for r in c['hot_threads'][:4]])"
  done
done
echo ALL_OK
