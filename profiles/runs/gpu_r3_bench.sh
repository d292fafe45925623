#!/usr/bin/env bash
# Round 3: GPU tests, then the headline bench (frontend entry, mTLS on) under the driver's flags,
# the same with mTLS off (A/B), and round 2's api-sidecar entry -- per-process CPU on stderr.
set -euo pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
nproc > gpurun_out/r3_host.txt; cat /sys/fs/cgroup/cpu.max >> gpurun_out/r3_host.txt 2>/dev/null || true
python - >> gpurun_out/r3_host.txt <<'PY'
import os; from aca_dotnet_workshop_amd.parallel import gpu_numa_nodes, host_topology
print("affinity", len(os.sched_getaffinity(0)), "gpu_numa", gpu_numa_nodes(), "nodes", [len(n) for n in host_topology()[0]])
PY
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3_pytest_gpu.log 2>&1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_fe.json 2> gpurun_out/r3_bench_fe.err
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --mtls 0 > gpurun_out/r3_bench_fe_nomtls.json 2> gpurun_out/r3_bench_fe_nomtls.err
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --entry api-sidecar > gpurun_out/r3_bench_api.json 2> gpurun_out/r3_bench_api.err
echo ALL_OK
