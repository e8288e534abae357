#!/bin/bash
# Parity + c3 bench + round profiles (under gpurun).
set -o pipefail
O=gpurun_out/final
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_fate.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 240 python bench.py --no-cpu-baseline --no-decode-check > $O/c3.json 2> $O/c3.err || exit 2
bash tools/profile_round.sh r02 --steps 5 || exit 3
bash tools/profile_round.sh r02_c4 --config c4 --steps 5 || exit 4
echo done
