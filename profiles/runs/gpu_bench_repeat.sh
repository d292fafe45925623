#!/usr/bin/env bash
# Default bench, three times back to back (run-to-run spread on one box).
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd "$(dirname "$0")/../.."
rm -f gpurun_out/rep_*
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py > gpurun_out/rep_$i.json 2> gpurun_out/rep_$i.err
done
echo ALL_OK
