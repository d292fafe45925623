#!/usr/bin/env bash
# PMC counters for the query kernels (own runs: counters + kernel trace only), then the
# end-to-end 10M-doc state query with the default (two-pass) select.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd "$(dirname "$0")/../.."
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc1 -o q -- python3 bench_query.py --rows 100000000 --iters 3 --warmup 1 > gpurun_out/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc2 -o q -- python3 bench_query.py --rows 100000000 --iters 3 --warmup 1 > gpurun_out/pmc2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc3 -o q -- python3 bench_query.py --rows 100000000 --iters 3 --warmup 1 > gpurun_out/pmc3.log 2>&1
timeout -k 10 600 python bench_query_e2e.py --docs 10000000 --accel gpu --queries 30 > gpurun_out/qe2e_gpu_10m.json 2> gpurun_out/qe2e_gpu_10m.err
echo ALL_OK
