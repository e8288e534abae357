#!/bin/bash
# Host-frame pipeline: its parity tests, the PCIe-inclusive rates; then
# kernel timelines of the c3 bench: default, one records set, serial.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "encode2 or host_encode or avcodec or never_truncates or overflow" > $O/parity.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_alpha.py tests/test_v4.py > $O/alpha.log 2>&1 || exit 6
timeout -k 10 600 python tools/bench_host.py 21 10 $O/host_rates.json > $O/host.log 2>&1 || exit 2
bash tools/gpu_timeline.sh r3f_def --steps 6 || exit 3
FFV1HIP_RECSETS=1 bash tools/gpu_timeline.sh r3f_rec1 --steps 6 || exit 4
FFV1HIP_SERIAL=1 bash tools/gpu_timeline.sh r3f_serial --steps 4 || exit 5
echo done
