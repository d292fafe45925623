#!/usr/bin/env bash
# Round 4 baseline: the round-3 tree's headline under the driver's flags, then a shorter run
# with every process under cProfile (TT_PROFILE_DIR) for the by-function cost of the frontend
# and API app hops.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4base
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r4base/bench.json 2> gpurun_out/r4base/bench.err
echo "bench done"
TT_PROFILE_DIR=/tmp/r4prof timeout -k 10 600 python bench.py --steps 8 --warmup 2 --direct-steps 0 \
  > gpurun_out/r4base/bench_prof.json 2> gpurun_out/r4base/bench_prof.err
echo "profiled bench done"
for m in tasksmanager-frontend-webapp tasksmanager-backend-api tasksmanager-backend-processor; do
  python -m aca_dotnet_workshop_amd.telemetry.profiler /tmp/r4prof --match "$m" --top 45 --sort tottime \
    > "gpurun_out/r4base/prof_${m}.txt" || true
  python -m aca_dotnet_workshop_amd.telemetry.profiler /tmp/r4prof --match "$m" --top 45 --sort cumulative \
    > "gpurun_out/r4base/prof_${m}_cum.txt" || true
done
ls -la /tmp/r4prof > gpurun_out/r4base/prof_files.txt
echo ALL_OK
