#!/usr/bin/env bash
# Round 4: the sweep's mark half in one markoverdue call (the reference's form, MarkChunk=0) vs
# concurrent calls of at most 256 tasks spread over the API replicas (the default), alternated.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
out=gpurun_out/${R4MC_OUT:-r4mc}
mkdir -p $out
for i in 1 2; do
  for mc in ${R4MC_SIZES:-256 0}; do
    OverdueTasks__MarkChunk=$mc timeout -k 10 400 python bench.py --steps 20 --warmup 5 --envelope-s 0 --direct-steps 0 > $out/bench_${mc}_$i.json 2> $out/bench_${mc}_$i.err
    python -c "import json;d=json.load(open('$out/bench_${mc}_$i.json'));c=d['config'];s=c['overdue_sweeps'];t=s['trace']['spans_p50_ms'];print('markchunk=$mc', d['value'], c['cpu_us_per_task']['total'], s['sweep_p50_ms'], s['sweep_max_ms'], s['sweep_ms'], s['tasks_marked_overdue'], round(s['query_ms_total']/max(1,s['sweeps']),1), round(s['mark_ms_total']/max(1,s['sweeps']),1))"
  done
done
echo ALL_OK
