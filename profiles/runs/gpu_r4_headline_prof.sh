#!/usr/bin/env bash
# Round 4: kernel trace of the headline (driver's flags, no envelope) on the final tree: which
# HIP kernels the overdue sweep and the mirror's background sync run under load, and for how long.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
out=gpurun_out/${R4HP_OUT:-r4hprof}
mkdir -p $out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o bench -- python3 bench.py --steps 20 --warmup 5 --envelope-s 0 --direct-steps 0 > $out/bench.json 2> $out/bench.err
python3 -c "import json;d=json.load(open('$out/bench.json'));c=d['config'];s=c['overdue_sweeps'];print('bench', d['value'], c['cpu_us_per_task']['total'], s['sweep_p50_ms'], s['sweep_max_ms'], s['sweeps'])"
find $out/prof -name '*kernel_stats.csv' | while read f; do echo "== $f"; head -25 "$f"; done
echo ALL_OK
