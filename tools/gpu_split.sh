#!/bin/bash
# Walk part B priority sweep (under gpurun).
set -o pipefail
O=gpurun_out/prioB
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-decode-check"
run() { local tag=$1; shift; timeout -k 10 240 env "$@" $B $EXTRA > $O/$tag.json 2> $O/$tag.err || exit 1; }
EXTRA="" run b2 FFV1HIP_WALK_PRIO_B=2
EXTRA="" run b0 FFV1HIP_WALK_PRIO_B=0
EXTRA="" run b0c1 FFV1HIP_WALK_PRIO_B=0 FFV1HIP_CODE_WAVE_PRIO=1
EXTRA="" run b1c1 FFV1HIP_WALK_PRIO_B=1 FFV1HIP_CODE_WAVE_PRIO=1
echo done
