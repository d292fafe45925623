#!/usr/bin/env bash
# Round 4: where the native executables' CPU goes under the headline (TT_PC_SAMPLE self-profiles:
# own code vs each shared library vs each system call; native/src/pcsample.hpp).
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
out=$PWD/gpurun_out/${R4PC_OUT:-r4pcs}
mkdir -p $out/pcs
TT_PC_SAMPLE=$out/pcs/prof timeout -k 10 400 python bench.py --steps 20 --warmup 5 --envelope-s 0 --direct-steps 0 > $out/bench.json 2> $out/bench.err
python -c "import json;d=json.load(open('$out/bench.json'));c=d['config'];print('bench', d['value'], c['cpu_us_per_task']['total'])"
sleep 2
for f in $(ls -S $out/pcs | head -2) $(grep -l "== ingress" $out/pcs/* | head -1 | xargs -n1 basename); do
  head -50 $out/pcs/$f
done
echo ALL_OK
