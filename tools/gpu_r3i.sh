#!/bin/bash
# Round 3: host-frame path timing breakdown (FFV1HIP_HOSTDBG), copy-out on a
# thread of its own vs on the main thread, and the host memcpy ceiling.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 120 python tools/pcie_probe.py > $O/pcie.log 2>&1 || exit 1
FFV1HIP_HOSTDBG=1 timeout -k 10 600 python tools/bench_host.py 21 10 $O/host_async.json > $O/host_async.log 2>&1 || exit 2
FFV1HIP_HOSTDBG=1 FFV1HIP_COPYOUT_SYNC=1 timeout -k 10 600 python tools/bench_host.py 21 10 $O/host_sync.json > $O/host_sync.log 2>&1 || exit 3
echo done
