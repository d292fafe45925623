#!/usr/bin/env bash
# A/B of the services' HTTP host on one box: pure-Python asyncio I/O vs the native app host
# (apphost.hpp) for server+client, server only, client only.  Same build, back to back.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd "$(dirname "$0")/../.."
for i in 1 2 3; do
  for mode in python native; do
    timeout -k 10 300 python bench.py --steps 40 --warmup 5 --app-host "$mode" > gpurun_out/ab_${mode}_$i.json 2> gpurun_out/ab_${mode}_$i.err
  done
done
echo ALL_OK
