#!/bin/bash
# Long-stream coder waves above the walk: threshold sweep (under gpurun).
set -o pipefail
O=gpurun_out/boost
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-decode-check"
run() { local tag=$1; shift; timeout -k 10 240 env "$@" $B $EXTRA > $O/$tag.json 2> $O/$tag.err || exit 1; }
EXTRA="" run off FFV1HIP_CODE_BOOST=0
EXTRA="" run b100 FFV1HIP_CODE_BOOST=100
EXTRA="" run b120 FFV1HIP_CODE_BOOST=120
EXTRA="" run b140 FFV1HIP_CODE_BOOST=140
EXTRA="--config c4" run c4_b120 FFV1HIP_CODE_BOOST=120
EXTRA="--config c4" run c4_off FFV1HIP_CODE_BOOST=0
echo done
