#!/bin/bash
# Schedule fix (the batch's kernels on internal streams): parity, bench, timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $O/parity.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > $O/bench.json 2> $O/bench.err || exit 2
bash tools/gpu_timeline.sh r3d --steps 6 || exit 3
echo done
