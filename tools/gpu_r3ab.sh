#!/bin/bash
# Round 3 final lines: GPU suite with the per-batch priority rule, then
# c3 (the driver's command), c2, c4 (19 GOPs), c5 (5 GOPs) with the CPU
# baseline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3ab
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $O/gpu.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_c3.json 2> $O/b_c3.err || exit 2
for c in c2 c4 c5; do
  timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 2 > $O/b_$c.json 2> $O/b_$c.err || exit 3
done
echo done
