#!/bin/bash
# round 6: requests in flight (the load generator's concurrency) on the final tree, headline only,
# alternating 192 (default) / 256 / 320
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6conc
mkdir -p $out
run() {
  local tag=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --alt-steps 0 --envelope-s 0 --keda-messages 0 \
    --ingest-messages 0 --session-flows 0 --browser-steps 0 --direct-steps 0 "$@" > $out/$tag.json 2> $out/$tag.err
}
run c192a --concurrency 192 && run c256a --concurrency 256 && run c320a --concurrency 320 && \
  run c192b --concurrency 192 && run c256b --concurrency 256 && run c320b --concurrency 320 || exit $?
exit 0
