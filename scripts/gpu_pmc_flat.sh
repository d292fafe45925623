#!/usr/bin/env bash
# PMC counters for tt_scan_eval_t<2> vs tt_scan_flat_t (bench_query runs both): is the scan
# instruction- or memory-bound?  One counter pass per run (no trace domains with --pmc).
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd "$(dirname "$0")/.."
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmcf1 -o q -- python3 bench_query.py --rows 100000000 --iters 3 --warmup 1 > gpurun_out/pmcf1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcf2 -o q -- python3 bench_query.py --rows 100000000 --iters 3 --warmup 1 > gpurun_out/pmcf2.log 2>&1
echo ALL_OK
