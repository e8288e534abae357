#!/bin/bash
# Round 3: the new dense-rows test; c4 / c2 / c5 at their batches (with the
# CPU baseline), c4 and c2 with the round-2 wave priorities (walk 2, range
# 0); the --gpus 2 launch on one device; host rates.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3aa
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "dense_rows or state_forwarding" > $O/parity.log 2>&1 || exit 1
run() {  # tag env args...
  local tag=$1 env=$2; shift 2
  env $env timeout -k 10 400 python bench.py "$@" > $O/b_$tag.json 2> $O/b_$tag.err
}
run c4_19 "" --config c4 --gops 19 --steps 10 --warmup 2 || exit 2
run c4_16p "FFV1HIP_WALK_PRIO=2 FFV1HIP_RANGE_PRIO=0" --config c4 --gops 16 --steps 10 --warmup 2 --no-cpu-baseline || exit 3
run c4_19p "FFV1HIP_WALK_PRIO=2 FFV1HIP_RANGE_PRIO=0" --config c4 --gops 19 --steps 10 --warmup 2 --no-cpu-baseline || exit 4
run c2p "FFV1HIP_WALK_PRIO=2 FFV1HIP_RANGE_PRIO=0" --config c2 --steps 10 --warmup 2 --no-cpu-baseline || exit 5
run c5_5 "" --config c5 --gops 5 --steps 10 --warmup 2 || exit 6
run c5_6 "" --config c5 --gops 6 --steps 10 --warmup 2 --no-cpu-baseline || exit 7
FFV1_BENCH_ONE_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --gops 6 --steps 5 --no-cpu-baseline > $O/b_2rank.json 2> $O/b_2rank.err || exit 8
timeout -k 10 400 python bench.py --gops 6 --steps 5 --no-cpu-baseline > $O/b_1rank6.json 2> $O/b_1rank6.err || exit 9
FFV1HIP_HOSTDBG=1 timeout -k 10 600 python tools/bench_host.py 20 10 $O/host_rates.json > $O/host.log 2>&1 || exit 10
echo done
