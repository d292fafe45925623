#!/bin/bash
# top-k phase clocks (stamps) + kernel trace of the same runs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_columnar.py -m gpu -k "topk or select or page or zone" > gpurun_out/r3v_tests.log 2>&1 &&
timeout -k 10 120 python -u scripts/topk_phases.py --out gpurun_out/r3v_topk_phases.json > gpurun_out/r3v_phases.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r3v_prof -o run -- python3 scripts/topk_phases.py > gpurun_out/r3v_prof.log 2>&1
rc=$?
tail -3 gpurun_out/r3v_tests.log; cat gpurun_out/r3v_phases.log
exit $rc
