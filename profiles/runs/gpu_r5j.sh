#!/bin/bash
# round 5: the driver's command after the pipelined connections, then a kernel trace and PC samples
# rocprofv3 kernel trace of a shorter headline run and the data plane's PC samples
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5j
mkdir -p $out/pcs
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 20 --warmup 5 \
  --envelope-s 0 --direct-steps 0 --browser-steps 0 > $out/prof_bench.json 2> $out/prof_bench.err || exit $?
TT_PC_SAMPLE=$PWD/$out/pcs/prof timeout -k 10 300 python bench.py --steps 20 --warmup 5 --envelope-s 0 \
  --direct-steps 0 --browser-steps 0 > $out/pcs_bench.json 2> $out/pcs_bench.err
