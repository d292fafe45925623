#!/usr/bin/env bash
# Round 4: GPU tests after the markoverdue / bulk-get / TLS read-loop changes, then the ingress
# A/B again (ingress over the replicas' Unix sockets, TLS short-record reads).
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r4ab2
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4ab2/pytest_gpu.log 2>&1
tail -3 gpurun_out/r4ab2/pytest_gpu.log
R4AB_OUT=r4ab2 bash profiles/runs/gpu_r4_ingress_ab.sh
