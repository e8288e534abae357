#!/bin/bash
# Bits kernel placement under the split schedule (under gpurun).
set -o pipefail
O=gpurun_out/bitsplace
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "split or config3" > $O/tests.log 2>&1 || exit 1
B="python bench.py --no-cpu-baseline --no-decode-check"
run() { local tag=$1; shift; timeout -k 10 240 env "$@" $B $EXTRA > $O/$tag.json 2> $O/$tag.err || exit 1; }
EXTRA="" run side FFV1HIP_BITS=side
EXTRA="" run code FFV1HIP_BITS=code
EXTRA="--config c5" run c5code FFV1HIP_BITS=code
EXTRA="--config c2" run c2code FFV1HIP_BITS=code
echo done
