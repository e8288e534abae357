#!/bin/bash
# Round 3 final: GPU suite and smoke on the final library, the driver's c3
# command, c2 / c4 / c5 lines (their PMC traffic now in profiles/).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3af
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $O/gpu.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_c3.json 2> $O/b_c3.err || exit 3
for c in c2 c4 c5; do
  timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 2 > $O/b_$c.json 2> $O/b_$c.err || exit 4
done
echo done
