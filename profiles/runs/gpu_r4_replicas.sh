#!/usr/bin/env bash
# Round 4: replica layouts (frontend:api:processor) with the native routes, alternated on one box.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
out=gpurun_out/${R4REP_OUT:-r4rep}
mkdir -p $out
for i in 1 2; do
  for lay in ${R4REP_LIST:-4:4:2 4:4:3 3:4:3 4:5:2}; do
    IFS=: read fe api proc <<< "$lay"
    tag=${lay//:/_}
    timeout -k 10 400 python bench.py --steps 20 --warmup 5 --envelope-s 0 --direct-steps 0 --frontend-replicas $fe --api-replicas $api --processor-replicas $proc ${R4REP_EXTRA:-} > $out/bench_${tag}_$i.json 2> $out/bench_${tag}_$i.err
    python -c "import json;d=json.load(open('$out/bench_${tag}_$i.json'));c=d['config'];u=c['cpu_us_per_task'];t=c['cpu_limits']['throttling_in_timed_region'];print('$lay', d['value'], u['total'], c['cpu_limits']['vcpu_per_replica'], c['create_latency_p50_ms'], c['create_latency_p99_ms'], c['overdue_sweeps']['sweep_p50_ms'], {k: v['stopped_share'] for k, v in t.items()})"
    grep -h -o '"total_cores_busy": [0-9.]*' $out/bench_${tag}_$i.err || true
  done
done
echo ALL_OK
