#!/bin/bash
# Round 3, final library: c3 on the D2 stress content (LSB-active noise) and
# the --gpus 2 launch rehearsed on one device.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3ah
mkdir -p $O
timeout -k 10 400 python bench.py --data d2 --steps 10 --warmup 2 --no-cpu-baseline > $O/b_d2.json 2> $O/b_d2.err || exit 1
FFV1_BENCH_ONE_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --gops 6 --steps 5 --no-cpu-baseline > $O/b_2rank.json 2> $O/b_2rank.err || exit 2
echo done
