#!/bin/bash
# Round 3: the other BASELINE configs (c2 1080p intra, c4 4K 4:4:4 12-bit,
# c5 8K) at their batch sizes with the CPU baseline; the --gpus 2 launch
# rehearsed on one device; host-frame rates.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3w
mkdir -p $O
timeout -k 10 400 python bench.py --config c2 --steps 10 --warmup 2 > $O/b_c2.json 2> $O/b_c2.err || exit 1
for g in 16 20; do
  timeout -k 10 400 python bench.py --config c4 --gops $g --steps 10 --warmup 2 > $O/b_c4_$g.json 2> $O/b_c4_$g.err || exit 2
done
for g in 5 6; do
  timeout -k 10 400 python bench.py --config c5 --gops $g --steps 10 --warmup 2 > $O/b_c5_$g.json 2> $O/b_c5_$g.err || exit 3
done
FFV1_BENCH_ONE_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --gops 6 --steps 5 --no-cpu-baseline > $O/b_2rank.json 2> $O/b_2rank.err || exit 4
timeout -k 10 400 python bench.py --gops 6 --steps 5 --no-cpu-baseline > $O/b_1rank6.json 2> $O/b_1rank6.err || exit 5
FFV1HIP_HOSTDBG=1 timeout -k 10 600 python tools/bench_host.py 20 10 $O/host_rates.json > $O/host.log 2>&1 || exit 6
echo done
