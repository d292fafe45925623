#!/usr/bin/env bash
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 15 --app-host native > gpurun_out/w15_native_$i.json 2> gpurun_out/w15_native_$i.err
done
echo ALL_OK
