#!/bin/bash
# Partial split (one records set): GPU suite, then c4 / c3 benches (under gpurun).
set -o pipefail
O=gpurun_out/part
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || exit 1
B="python bench.py --no-cpu-baseline"
run() { local tag=$1; shift; timeout -k 10 300 env "$@" $B $EXTRA > $O/$tag.json 2> $O/$tag.err || exit 1; }
EXTRA="--config c4" run c4 FFV1HIP_PARTIAL=1
EXTRA="--config c4" run c4_off FFV1HIP_PARTIAL=0
EXTRA="--no-decode-check" run c3_one FFV1HIP_RECSETS=1
EXTRA="--no-decode-check" run c3 FFV1HIP_RECSETS=2
echo done
