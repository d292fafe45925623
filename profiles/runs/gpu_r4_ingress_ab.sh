#!/usr/bin/env bash
# Round 4: headline with load entering at the frontend's native external HTTPS ingress vs the
# ingress bypassed (load balanced over the frontend replicas), alternated on one box; plus one
# run through the asyncio ingress for scale.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
out=gpurun_out/${R4AB_OUT:-r4ab}
mkdir -p $out
for i in 1 2 3; do
  for mode in native bypass; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --ingress $mode --direct-steps 0 \
      > $out/bench_${mode}_$i.json 2> $out/bench_${mode}_$i.err
    echo "$mode $i: $(python -c "import json;d=json.load(open('$out/bench_${mode}_$i.json'));print(d['value'], d['config']['cpu_us_per_task']['total'])")"
  done
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --ingress python --direct-steps 0 \
  > $out/bench_python_1.json 2> $out/bench_python_1.err
echo "python: $(python -c "import json;d=json.load(open('$out/bench_python_1.json'));print(d['value'])")"
echo ALL_OK
