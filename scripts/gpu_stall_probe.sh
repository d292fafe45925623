#!/usr/bin/env bash
# Native-app-host bench runs with hand-off tracing (TT_STALL_LOG) and GC pause logging
# (TT_GC_LOG) in every process, to locate latency stalls.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd "$(dirname "$0")/.."
rm -f gpurun_out/stall*.log gpurun_out/gc*.log
for i in 1 2; do
  TT_GC_LOG=$PWD/gpurun_out/gc_$i.log TT_STALL_LOG=$PWD/gpurun_out/stall_$i.log timeout -k 10 300 python bench.py --steps 40 --warmup 5 --app-host native > gpurun_out/stall_bench_$i.json 2> gpurun_out/stall_bench_$i.err
done
echo ALL_OK
