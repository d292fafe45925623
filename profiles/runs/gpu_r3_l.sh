#!/usr/bin/env bash
# Round 3 (l): what the per-replica CPU caps cost the headline and the sweep -- default (20 ms
# duty cycle), a 10 ms duty cycle, and no caps -- back to back on one box.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3l_caps20.json 2> gpurun_out/r3l_caps20.err
TT_CPU_PERIOD_MS=10 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3l_caps10.json 2> gpurun_out/r3l_caps10.err
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --cpu-limits 0 > gpurun_out/r3l_nocaps.json 2> gpurun_out/r3l_nocaps.err
echo ALL_OK
