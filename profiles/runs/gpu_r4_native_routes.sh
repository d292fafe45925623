#!/usr/bin/env bash
# Round 4: the app host's native routes (frontend POST /Tasks/Create, API POST /api/tasks) vs
# the Python handlers (TT_NATIVE_ROUTES=0), alternated on one box under the driver's flags; then
# the GPU tests.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
out=gpurun_out/${R4NR_OUT:-r4nr}
mkdir -p $out
for i in 1 2; do
  for nr in 1 0; do
    TT_NATIVE_ROUTES=$nr timeout -k 10 400 python bench.py --steps 20 --warmup 5 --envelope-s 0 > $out/bench_${nr}_$i.json 2> $out/bench_${nr}_$i.err
    python -c "import json;d=json.load(open('$out/bench_${nr}_$i.json'));c=d['config'];s=c['overdue_sweeps'];u=c['cpu_us_per_task'];print('native_routes=$nr', d['value'], u['total'], u['apps_frontend_plus_api'], {k: v for k, v in u['by_role'].items() if k.endswith('.app')}, s['sweep_p50_ms'], s['sweep_max_ms'], c['api_sidecar_direct']['value'], c['create_latency_p50_ms'], c['create_latency_p99_ms'])"
  done
done
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
tail -2 $out/pytest_gpu.log
echo ALL_OK
