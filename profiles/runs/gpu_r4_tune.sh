#!/usr/bin/env bash
# Round 4: with the native routes on, what bounds the headline? Variants alternated on one box
# (driver's flags, no envelope): replica layouts, ingress event loops, backing front threads,
# and a no-sweep control.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
out=gpurun_out/${R4TUNE_OUT:-r4tune}
mkdir -p $out
run() {  # tag, env assignments..., -- bench args...
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 400 python bench.py --steps 20 --warmup 5 --envelope-s 0 --direct-steps 0 "$@" > $out/$tag.json 2> $out/$tag.err
  python -c "import json;d=json.load(open('$out/$tag.json'));c=d['config'];u=c['cpu_us_per_task'];t=c['cpu_limits']['throttling_in_timed_region'];s=c['loadgen']['steps_ms'] if 'steps_ms' in c.get('loadgen',{}) else [];print('$tag', d['value'], u['total'], c['replicas'], c['create_latency_p50_ms'], c['create_latency_p99_ms'], c['overdue_sweeps'].get('sweep_p50_ms'), {k: v['stopped_share'] for k, v in t.items()})"
  grep -h -o '"total_cores_busy": [0-9.]*' $out/$tag.err || true
}
for i in 1 2; do
  run base_$i X=1 -- 
  run api5_$i X=1 -- --api-replicas 5
  run fe3proc3_$i X=1 -- --frontend-replicas 3 --processor-replicas 3
  run ing4_$i TT_INGRESS_THREADS=4 --
  run bf4_$i TT_BACKING_FRONT_THREADS=4 --
  run lg2_$i X=1 -- --loadgen-threads 2
done
run nosweep X=1 -- --overdue-sweep-ms 0
echo ALL_OK
