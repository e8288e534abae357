#!/bin/bash
# Decoder iteration (under gpurun): GPU suite, then the c3 bench's decode self-check with and without swap.
set -o pipefail
O=gpurun_out/dec
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > $O/c3.json 2> $O/c3.err || exit 2
timeout -k 10 300 env FFV1HIP_DEC_SWAP=0 python bench.py --no-cpu-baseline --steps 3 > $O/c3_noswap.json 2> $O/c3_noswap.err || exit 3
echo done
