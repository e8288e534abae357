#!/bin/bash
# Equal wave priorities; larger c3 batches with the split forced (under gpurun).
set -o pipefail
O=gpurun_out/prio5
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-decode-check --steps 10"
run() { local tag=$1; shift; timeout -k 10 240 env "$@" $B $EXTRA > $O/$tag.json 2> $O/$tag.err || exit 1; }
EXTRA="" run base FFV1HIP_WALK_PRIO=2
EXTRA="" run w1c1 FFV1HIP_WALK_PRIO=1 FFV1HIP_CODE_WAVE_PRIO=1
EXTRA="" run w2c2 FFV1HIP_CODE_WAVE_PRIO=2
EXTRA="" run w3c2 FFV1HIP_WALK_PRIO=3 FFV1HIP_CODE_WAVE_PRIO=2
EXTRA="--gops 22" run g22 FFV1HIP_SPLIT_MAX=95
EXTRA="--gops 23" run g23 FFV1HIP_SPLIT_MAX=95
echo done
