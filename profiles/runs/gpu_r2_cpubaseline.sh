#!/usr/bin/env bash
# Round 2: the GPU scan against the fair host baseline (native multi-threaded executor over the
# same narrow codes, the box's whole CPU share) -- kernel microbench at 1e8 rows and the state
# query through the full stack at 10M documents, GPU vs CPU columnar.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 400 python bench_query.py --rows 100000000 --iters 20 > gpurun_out/bq_fair.json 2> gpurun_out/bq_fair.err
timeout -k 10 600 python bench_query_e2e.py --docs 10000000 --accel cpu --queries 20 > gpurun_out/qe2e_cpu.json 2> gpurun_out/qe2e_cpu.err
timeout -k 10 600 python bench_query_e2e.py --docs 10000000 --accel gpu --queries 20 > gpurun_out/qe2e_gpu.json 2> gpurun_out/qe2e_gpu.err
echo ALL_OK
