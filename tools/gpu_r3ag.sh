#!/bin/bash
# Round 3: host-frame encode with the collector joined after the staging:
# the host-path GPU tests, then the host rates.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3ag
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_container.py tests/test_alpha.py tests/test_v4.py tests/test_gpu_twopass.py > $O/parity.log 2>&1 || exit 1
FFV1HIP_HOSTDBG=1 timeout -k 10 600 python tools/bench_host.py 20 10 $O/host_rates.json > $O/host.log 2>&1 || exit 2
echo done
