#!/usr/bin/env bash
# Round 3 (ab): three headline benches back to back, with a process / load snapshot between them
# (does a run leave anything behind that slows the next one?).
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
snap() {
  { date +%T; cat /proc/loadavg; ps -u "$(id -u)" -o pid,ppid,pcpu,rss,etime,comm --sort=-pcpu | head -25; } > "gpurun_out/r3ab_ps_$1.txt" 2>&1 || true
}
snap 0
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3ab_bench_1.json 2> gpurun_out/r3ab_bench_1.err
snap 1
sleep 5
snap 1b
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3ab_bench_2.json 2> gpurun_out/r3ab_bench_2.err
snap 2
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3ab_bench_3.json 2> gpurun_out/r3ab_bench_3.err
snap 3
echo ALL_OK
