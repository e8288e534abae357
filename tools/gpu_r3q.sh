#!/bin/bash
# Round 3: new defaults (symbols/bits/dseg bounded grids, the next batch's
# symbols from the start of the walk, 8-byte records): GPU suite, the
# driver's bench command, one walk launch vs two, host rates.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3q
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $O/gpu.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_def.json 2> $O/b_def.err || exit 2
FFV1HIP_WALK_SPLIT=0 FFV1HIP_WALKTRACE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 20 > $O/b_one.json 2> $O/b_one.err || exit 3
FFV1HIP_WALKTRACE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 20 > $O/b_two.json 2> $O/b_two.err || exit 4
FFV1HIP_HOSTDBG=1 timeout -k 10 600 python tools/bench_host.py 21 10 $O/host_rates.json > $O/host.log 2>&1 || exit 5
echo done
