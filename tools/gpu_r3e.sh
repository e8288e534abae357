#!/bin/bash
# Round 3 re-entry: the whole -m gpu suite, smoke(), the c3 bench (every GOP
# against the oracle fixture, CPU baseline), then the round profile
# (kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 3
bash tools/profile_round.sh r03 --steps 10 || exit 4
echo done
