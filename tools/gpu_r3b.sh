#!/bin/bash
# Round 3: the three-pass range coder: parity first, then the c3 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $O/parity.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > $O/bench.json 2> $O/bench.err || exit 2
echo done
