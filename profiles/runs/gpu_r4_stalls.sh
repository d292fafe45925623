#!/usr/bin/env bash
# Round 4: what stalls for 15+ ms during the headline (sweep outliers): loop gaps of every native
# loop, backing-services log write(2)s, Python GC pauses and slow app-host hand-offs.
set -euo pipefail
export TMPDIR=${R4ST_TMP:-/tmp}
cd "$(dirname "$0")/../.."
out=$PWD/gpurun_out/${R4ST_OUT:-r4st}
mkdir -p $out
for i in ${R4ST_RUNS:-1 2}; do
  TT_STALL_LOG=$out/stall_$i.jsonl TT_STALL_MS=15 TT_GC_LOG=$out/gc_$i.jsonl timeout -k 10 400 python bench.py --steps 20 --warmup 5 --envelope-s 0 --direct-steps 0 > $out/bench_$i.json 2> $out/bench_$i.err
  python -c "import json;d=json.load(open('$out/bench_$i.json'));c=d['config'];s=c['overdue_sweeps'];print('run $i', d['value'], c['cpu_us_per_task']['total'], s['sweep_p50_ms'], s['sweep_max_ms'], s['sweep_ms'])"
  touch $out/stall_$i.jsonl $out/gc_$i.jsonl
  wc -l $out/stall_$i.jsonl $out/gc_$i.jsonl
done
echo ALL_OK
