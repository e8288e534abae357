#!/bin/bash
# Kernel times with and without the two pipelines overlapping.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3c
mkdir -p $O
FFV1HIP_SERIAL=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 6 > $O/serial.json 2> $O/serial.err || exit 1
echo done
