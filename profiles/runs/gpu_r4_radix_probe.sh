#!/usr/bin/env bash
# Round 4: the onesweep radix pair sort alone (scripts/radix_probe.py): its GPU tests, sort-only
# timings at the query path's size, a kernel trace and one counter pass over the sort kernels.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
out=gpurun_out/${R4RADIX_OUT:-r4probe}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_columnar.py -x -q -m gpu -k "radix or ordered" --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
tail -2 $out/pytest.log
timeout -k 10 180 python scripts/radix_probe.py > $out/probe.json
timeout -k 10 180 python scripts/radix_probe.py --bits 63 --high-values 1000000000 >> $out/probe.json
timeout -k 10 180 python scripts/radix_probe.py --n 100000 --iters 200 >> $out/probe.json
timeout -k 10 180 python scripts/radix_probe.py --n 1000000 --iters 100 >> $out/probe.json
cat $out/probe.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o p -- python3 scripts/radix_probe.py --iters 5 > $out/prof.log 2>&1
echo traced
if [ -z "${R4RADIX_NOPMC:-}" ]; then
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR -d $out/pmc1 -o c -- python3 scripts/radix_probe.py --iters 2 --warmup 1 > $out/pmc1.log 2>&1
  echo pmc1
fi
echo ALL_OK
