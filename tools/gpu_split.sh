#!/bin/bash
# Wave priority sweep for the walk and the coder (under gpurun).
set -o pipefail
O=gpurun_out/prio4
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-decode-check --steps 10"
run() { local tag=$1; shift; timeout -k 10 240 env "$@" $B $EXTRA > $O/$tag.json 2> $O/$tag.err || exit 1; }
EXTRA="" run w2c0 FFV1HIP_WALK_PRIO=2
EXTRA="" run w2c3 FFV1HIP_CODE_WAVE_PRIO=3
EXTRA="" run w0c0 FFV1HIP_WALK_PRIO=0
EXTRA="" run w1c2 FFV1HIP_WALK_PRIO=1 FFV1HIP_CODE_WAVE_PRIO=2
EXTRA="" run w0c3 FFV1HIP_WALK_PRIO=0 FFV1HIP_CODE_WAVE_PRIO=3
echo done
