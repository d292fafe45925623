#!/bin/bash
# round 6: replica topology at the same CPU budget (headline only): does spreading the API's
# sidecar work over more data-plane loops lower the queueing per hop?
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6w
mkdir -p $out
run() {
  local tag=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --alt-steps 0 --envelope-s 0 --keda-messages 0 \
    --ingest-messages 0 --session-flows 0 --browser-steps 0 --direct-steps 0 "$@" > $out/$tag.json 2> $out/$tag.err
}
run base && run api6 --api-replicas 6 && run api6fe6 --api-replicas 6 --frontend-replicas 6 --concurrency 192 \
  && run api8 --api-replicas 8 && run base2 || exit $?
exit 0
