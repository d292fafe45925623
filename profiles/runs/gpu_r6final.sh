#!/bin/bash
# round 6 confirmation: GPU tests, the driver's smoke, the driver's bench command twice
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r6s}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/gputests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/bench$i.json 2> $out/bench$i.err || exit $?
done
