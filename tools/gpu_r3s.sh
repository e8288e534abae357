#!/bin/bash
# Round 3: one-wave bits blocks; dense rows at 21 and 20 GOPs per step
# (20 GOPs = 1280 walk waves = all resident at 5 per CU).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3s
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_fate.py tests/test_alpha.py tests/test_v4.py tests/test_gpu_twopass.py > $O/parity.log 2>&1 || exit 1
for v in ctx21 dense21 dense20 dense20s ctx20; do
  case $v in
    ctx21) E="FFV1HIP_DENSE=0"; G=21 ;;
    dense21) E=""; G=21 ;;
    dense20) E=""; G=20 ;;
    dense20s) E="FFV1HIP_WALK_SPLIT=0"; G=20 ;;
    ctx20) E="FFV1HIP_DENSE=0"; G=20 ;;
  esac
  env $E FFV1HIP_WALKTRACE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 20 --gops $G > $O/b_$v.json 2> $O/b_$v.err || exit 4
done
FFV1HIP_HOSTDBG=1 timeout -k 10 600 python tools/bench_host.py 21 10 $O/host_rates.json > $O/host.log 2>&1 || exit 6
echo done
