#!/usr/bin/env bash
# SURVEY §7.5 latency benchmarks on the box: 2-hop CRUD, publish->ack, time-to-scale.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd "$(dirname "$0")/.."
timeout -k 10 600 python bench_latency.py --ops 300 --events 300 > gpurun_out/latency.jsonl 2> gpurun_out/latency.err
echo ALL_OK
