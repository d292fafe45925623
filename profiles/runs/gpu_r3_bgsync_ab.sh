#!/usr/bin/env bash
# A/B: the backing's background mirror sync (default 100 ms) vs none, headline bench under the
# driver's flags: does the sync thread's GIL time delay the query page's way back?
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3bg_on.json 2> gpurun_out/r3bg_on.err
TT_QUERY_MIRROR_SYNC_MS=0 timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3bg_off.json 2> gpurun_out/r3bg_off.err
echo ALL_OK
