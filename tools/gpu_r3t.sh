#!/bin/bash
# Round 3: dense rows at 20 GOPs: the coder's range pass (the longest chain
# once the walk is one round) at a wave priority above the walk's; ctx21
# sanity with the 4-wave bits blocks back.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3t
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "c3 or batch or split or device" > $O/parity.log 2>&1 || exit 1
for v in ctx21 d20 d20r3 d20r3d3 d20r3s2 d21r3; do
  case $v in
    ctx21) E="FFV1HIP_DENSE=0"; G=21 ;;
    d20) E=""; G=20 ;;
    d20r3) E="FFV1HIP_RANGE_PRIO=3"; G=20 ;;
    d20r3d3) E="FFV1HIP_RANGE_PRIO=3 FFV1HIP_DSEG_PRIO=3"; G=20 ;;
    d20r3s2) E="FFV1HIP_RANGE_PRIO=3 FFV1HIP_SYM_GRID=2048 FFV1HIP_DSEG_GRID=2048"; G=20 ;;
    d21r3) E="FFV1HIP_RANGE_PRIO=3"; G=21 ;;
  esac
  env $E FFV1HIP_WALKTRACE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 20 --gops $G > $O/b_$v.json 2> $O/b_$v.err || exit 4
done
echo done
