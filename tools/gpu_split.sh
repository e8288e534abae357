#!/bin/bash
# Two coder streams: GPU suite, then benches with and without (under gpurun).
set -o pipefail
O=gpurun_out/split3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || exit 1
B="python bench.py --no-cpu-baseline --no-decode-check"
run() { local tag=$1; shift; timeout -k 10 240 env "$@" $B $EXTRA > $O/$tag.json 2> $O/$tag.err || exit 1; }
EXTRA="" run c3 FFV1HIP_CODERS=2
EXTRA="" run c3_one FFV1HIP_CODERS=1
EXTRA="--config c5" run c5 FFV1HIP_CODERS=2
EXTRA="--config c2" run c2 FFV1HIP_CODERS=2
echo done
