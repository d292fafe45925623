#!/bin/bash
# round 5: hardware counters of the sweep path's kernels over the page-plan probe (one pass:
# 4 SQ counters + FETCH_SIZE, within one pass's limits; kernel trace only, no other tracing)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5t
mkdir -p $out
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU FETCH_SIZE --kernel-trace \
  -d $out/pmc -o run -- python3 profiles/runs/page_plan_probe.py > $out/probe.txt 2> $out/probe.err
