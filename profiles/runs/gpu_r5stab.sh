#!/bin/bash
# round 5: the driver's command four more times on the round-end tree (run-to-run spread of the
# headline, CPU per task and the sweep), plus a probe of the box's kernel TLS support
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5stab
mkdir -p $out
(cat /proc/sys/net/ipv4/tcp_available_ulp; ls /sys/module | grep -x tls || echo "no tls module"; uname -r) > $out/ktls_probe.txt 2>&1 || true
for i in 1 2 3 4; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/bench_$i.json 2> $out/bench_$i.err || exit $?
done
