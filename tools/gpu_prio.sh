#!/bin/bash
# Where the bits kernel runs: side / code / inline (under gpurun).
set -o pipefail
O=gpurun_out/bits
mkdir -p $O
B="python bench.py --no-cpu-baseline --no-decode-check"
run() { local tag=$1; shift; timeout -k 10 240 env "$@" $B $EXTRA > $O/$tag.json 2> $O/$tag.err || exit 1; }
EXTRA="" run c3_code FFV1HIP_BITS=code
EXTRA="" run c3_side FFV1HIP_BITS=side
EXTRA="--config c4" run c4_code FFV1HIP_BITS=code
EXTRA="--config c4 --gops 16" run c4g16_code FFV1HIP_BITS=code
EXTRA="--config c4 --gops 16" run c4g16_inline FFV1HIP_BITS=inline
EXTRA="--config c5" run c5_code FFV1HIP_BITS=code
EXTRA="--config c2" run c2_code FFV1HIP_BITS=code
echo done
