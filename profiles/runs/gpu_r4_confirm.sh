#!/usr/bin/env bash
# Round 4 confirmation of the committed tree: every GPU test, smoke(), the headline twice under
# the driver's flags (with the reference-envelope block), and the 1e8-row ORDER BY timings.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
out=gpurun_out/${R4CONFIRM_OUT:-r4confirm}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
tail -2 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
echo smoke ok
for i in 1 2; do
  timeout -k 10 420 python bench.py --steps 20 --warmup 5 > $out/bench_$i.json 2> $out/bench_$i.err
  python -c "import json;d=json.load(open('$out/bench_$i.json'));c=d['config'];s=c['overdue_sweeps'];e=c.get('reference_envelope',{});print('bench', d['value'], c['cpu_us_per_task']['total'], s['sweep_p50_ms'], s['sweep_max_ms'], e.get('tasks_per_s'), e.get('store_429s'))"
done
timeout -k 10 300 python bench_query.py --rows 100000000 --iters 20 --sorted > $out/bench_query.json 2> $out/bench_query.err
cat $out/bench_query.json
echo ALL_OK
