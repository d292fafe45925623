#!/usr/bin/env bash
# Round 4: processor CPU headroom A/B. The cron sweep runs in the processor, whose replicas the
# duty cycle stopped 9-13 % of the timed region at weight 0.67 (caps sized to its per-task
# demand); 0.85 leaves it headroom. Alternated on one box, driver's flags, no envelope.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
out=gpurun_out/${R4PW_OUT:-r4pw}
mkdir -p $out
for i in 1 2; do
  for w in ${R4PW_WEIGHTS:-1.0:1.42:0.67 1.0:1.42:0.85}; do
    tag=${w//:/_}
    timeout -k 10 400 python bench.py --steps 20 --warmup 5 --envelope-s 0 --cpu-weights $w > $out/bench_${tag}_$i.json 2> $out/bench_${tag}_$i.err
    python -c "import json;d=json.load(open('$out/bench_${tag}_$i.json'));c=d['config'];s=c['overdue_sweeps'];t=c['cpu_limits']['throttling_in_timed_region'];print('$w', d['value'], c['cpu_us_per_task']['total'], c['cpu_limits']['vcpu_per_replica'], s['sweep_p50_ms'], s['sweep_max_ms'], s['sweep_ms'], {k: v['stopped_share'] for k, v in t.items()})"
  done
done
echo ALL_OK
