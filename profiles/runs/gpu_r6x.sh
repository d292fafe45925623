#!/bin/bash
# round 6: fixed 4 MB TCP buffers on the sidecar mesh and the ingress (TT_TCP_BUF_KB) against the
# kernel's autotuning, alternating, headline only
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6x
mkdir -p $out
run() {
  local tag=$1 kb=$2
  TT_TCP_BUF_KB=$kb timeout -k 10 300 python bench.py --steps 20 --warmup 5 --alt-steps 0 --envelope-s 0 \
    --keda-messages 0 --ingest-messages 0 --session-flows 0 --browser-steps 0 --direct-steps 0 \
    > $out/$tag.json 2> $out/$tag.err
}
run a1 0 && run b1 4096 && run a2 0 && run b2 4096 && run a3 0 && run b3 4096 || exit $?
exit 0
