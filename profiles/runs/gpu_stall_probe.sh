#!/usr/bin/env bash
# Bench runs with stall tracing (TT_STALL_LOG: native host hand-offs, loop gaps of the app host,
# data planes and backing front) and GC pause logging (TT_GC_LOG); kernel memory-pressure
# counters (/proc/vmstat reclaim/compaction stalls, PSI) sampled around each run.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd "$(dirname "$0")/../.."
rm -f gpurun_out/stall*.log gpurun_out/gc*.log gpurun_out/vm_*.txt
snap() { { date +%s.%N; grep -E '^(allocstall|compact_stall|compact_fail|pgscan_direct|pgsteal_direct|thp_fault_alloc|thp_collapse_alloc|pgmajfault)' /proc/vmstat || true; cat /proc/pressure/memory 2>/dev/null || true; cat /proc/pressure/cpu 2>/dev/null || true; grep -E '^(MemFree|MemAvailable|AnonHugePages)' /proc/meminfo; cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag 2>/dev/null || true; } >> "$1"; }
for mode in native python native; do
  snap gpurun_out/vm_$mode.txt
  TT_GC_LOG=$PWD/gpurun_out/gc_$mode.log TT_STALL_LOG=$PWD/gpurun_out/stall_$mode.log timeout -k 10 300 python bench.py --steps 40 --warmup 5 --app-host $mode > gpurun_out/stall_bench_$mode.json 2> gpurun_out/stall_bench_$mode.err
  snap gpurun_out/vm_$mode.txt
done
echo ALL_OK
