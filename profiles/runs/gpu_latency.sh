#!/usr/bin/env bash
# SURVEY §7.5 latency benchmarks on the box (2-hop CRUD, publish->ack, time-to-scale) and the
# state query through the stack at 10M documents.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd "$(dirname "$0")/../.."
timeout -k 10 600 python bench_latency.py --ops 300 --events 300 > gpurun_out/latency.jsonl 2> gpurun_out/latency.err
timeout -k 10 600 python bench_query_e2e.py --docs 10000000 --accel gpu --queries 30 > gpurun_out/qe2e_10m.json 2> gpurun_out/qe2e_10m.err
echo ALL_OK
