#!/bin/bash
# Round 3: dense context rows in the walk's LDS above 8 bits (5 walk waves
# per CU), host path collecting batches with one D2H copy: GPU suite, c3
# dense vs context rows (walk trace), host rates.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3r
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $O/gpu.log 2>&1 || exit 1
FFV1HIP_WALKTRACE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 20 > $O/b_dense.json 2> $O/b_dense.err || exit 2
FFV1HIP_DENSE=0 FFV1HIP_WALKTRACE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 20 > $O/b_ctx.json 2> $O/b_ctx.err || exit 3
FFV1HIP_WALK_SPLIT=0 FFV1HIP_WALKTRACE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 20 > $O/b_dense1.json 2> $O/b_dense1.err || exit 4
FFV1HIP_WALKDBG=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 2 > $O/b_dbg.json 2> $O/b_dbg.err || exit 5
FFV1HIP_HOSTDBG=1 timeout -k 10 600 python tools/bench_host.py 21 10 $O/host_rates.json > $O/host.log 2>&1 || exit 6
echo done
