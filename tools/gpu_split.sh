#!/bin/bash
# Split walk schedule: benches of every config (under gpurun).
set -o pipefail
O=gpurun_out/split2
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-decode-check"
run() { local tag=$1; shift; timeout -k 10 240 env "$@" $B $EXTRA > $O/$tag.json 2> $O/$tag.err || exit 1; }
EXTRA="" run c3 FFV1HIP_RECSETS=2
EXTRA="--config c5" run c5 FFV1HIP_RECSETS=2
EXTRA="--config c2" run c2 FFV1HIP_RECSETS=2
EXTRA="--config c4" run c4 FFV1HIP_RECSETS=2
EXTRA="--data d2" run c3d2 FFV1HIP_RECSETS=2
echo done
