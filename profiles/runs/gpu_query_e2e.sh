#!/usr/bin/env bash
# State-query latency through the full stack: GPU accelerator vs CPU columnar vs native engine scan.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd "$(dirname "$0")/../.."
timeout -k 10 600 python bench_query_e2e.py --docs 10000000 --accel gpu --queries 20 > gpurun_out/qe2e_gpu_10m.json 2> gpurun_out/qe2e_gpu_10m.err
timeout -k 10 600 python bench_query_e2e.py --docs 10000000 --accel cpu --queries 10 > gpurun_out/qe2e_cpu_10m.json 2> gpurun_out/qe2e_cpu_10m.err
timeout -k 10 900 python bench_query_e2e.py --docs 2000000 --accel off --queries 3 > gpurun_out/qe2e_off_2m.json 2> gpurun_out/qe2e_off_2m.err
echo ALL_OK
