#!/usr/bin/env bash
# Round 3 (n): replica / concurrency sweep of the headline (one thread per core, the default).
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
run() { local tag=$1; shift; timeout -k 10 600 python bench.py --steps 20 --warmup 5 --direct-steps 0 "$@" > gpurun_out/r3n_$tag.json 2> gpurun_out/r3n_$tag.err; }
run base
run fe4_api5 --api-replicas 5
run fe3_api4 --frontend-replicas 3
run fe5_api5 --frontend-replicas 5 --api-replicas 5
run c256 --concurrency 256
run c128 --concurrency 128
run proc3 --processor-replicas 3
echo ALL_OK
