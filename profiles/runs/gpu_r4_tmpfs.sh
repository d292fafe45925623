#!/usr/bin/env bash
# Round 4: sweep outliers vs where the environment's state lives (backing-services append logs):
# the box's /tmp vs tmpfs (/dev/shm), alternated; prints the filesystem types first.
set -euo pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/${R4FS_OUT:-r4fs}
mkdir -p $out
df -hT /tmp /dev/shm | tee $out/df.txt
for i in 1 2; do
  for d in /dev/shm /tmp; do
    tag=$(basename $d)
    TMPDIR=$d timeout -k 10 400 python bench.py --steps 20 --warmup 5 --envelope-s 0 --direct-steps 0 > $out/bench_${tag}_$i.json 2> $out/bench_${tag}_$i.err
    python -c "import json;d=json.load(open('$out/bench_${tag}_$i.json'));c=d['config'];s=c['overdue_sweeps'];print('$tag', d['value'], c['cpu_us_per_task']['total'], s['sweep_p50_ms'], s['sweep_max_ms'], s['sweep_ms'], round(s['query_ms_total']/max(1,s['sweeps']),1), round(s['mark_ms_total']/max(1,s['sweeps']),1))"
  done
done
echo ALL_OK
