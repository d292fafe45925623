#!/usr/bin/env bash
# Round 2: SURVEY §7.5 latency benchmarks on the final tree (2-hop CRUD, publish -> ack, time-to-scale).
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python bench_latency.py --ops 300 --events 300 > gpurun_out/r2_latency.jsonl 2> gpurun_out/r2_latency.err
echo ALL_OK
