#!/bin/bash
# Round 3 final c3 line and profile: GPU suite, the driver's bench command,
# rocprofv3 kernel stats + PMC FETCH_SIZE / WRITE_SIZE of the same bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3y
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $O/gpu.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 2
timeout -k 10 1200 bash tools/profile_round.sh r03 --steps 10 > $O/prof.log 2>&1 || exit 3
echo done
