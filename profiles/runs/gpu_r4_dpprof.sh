#!/usr/bin/env bash
# Round 4: gprof of the sidecar data plane under the headline (a -pg build of dataplane.cpp
# selected with TT_DATAPLANE_BIN; one gmon file per data-plane process, flat profiles of the
# busiest four -- the API replicas' sidecars).
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
out=$PWD/gpurun_out/${R4DP_OUT:-r4dpprof}
mkdir -p $out/gmon
exe=$PWD/aca_dotnet_workshop_amd/native/bin/ttsidecar-dataplane-pg
TT_DATAPLANE_BIN=$exe GMON_OUT_PREFIX=$out/gmon/dp timeout -k 10 400 python bench.py --steps 20 --warmup 5 --envelope-s 0 --direct-steps 0 > $out/bench.json 2> $out/bench.err
python -c "import json;d=json.load(open('$out/bench.json'));c=d['config'];print('bench', d['value'], c['cpu_us_per_task']['total'], c['cpu_us_per_task']['by_role'])"
ls -S $out/gmon | head -4 > $out/top.txt
n=0
for f in $(cat $out/top.txt); do
  n=$((n+1))
  gprof -b -p $exe $out/gmon/$f > $out/flat_$n.txt
  head -45 $out/flat_$n.txt
done
rm -rf $out/gmon
echo ALL_OK
