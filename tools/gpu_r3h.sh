#!/bin/bash
# Round 3: the walk's shader clock (s_memtime over s_memrealtime per wave)
# with the coder beside it and alone (FFV1HIP_SERIAL), the serial kernel
# timeline, the PCIe ceiling and the host-frame rates.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3h
mkdir -p $O
FFV1HIP_WALKDBG=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 6 > $O/dbg_def.json 2> $O/dbg_def.err || exit 1
FFV1HIP_WALKDBG=1 FFV1HIP_SERIAL=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 6 > $O/dbg_serial.json 2> $O/dbg_serial.err || exit 2
FFV1HIP_SERIAL=1 bash tools/gpu_timeline.sh r3h_serial --steps 4 || exit 3
timeout -k 10 120 python tools/pcie_probe.py > $O/pcie.log 2>&1 || exit 4
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "host_encode or encode2 or avcodec" > $O/parity.log 2>&1 || exit 5
timeout -k 10 600 python tools/bench_host.py 21 10 $O/host_rates.json > $O/host.log 2>&1 || exit 6
echo done
