#!/bin/bash
# Round 3: dense rows at 20 GOPs, wave priorities of walk / range and the
# side grids.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3u
mkdir -p $O
for v in d20r3 w0 w0r1 w1r3 r3big w0r3; do
  case $v in
    d20r3) E="FFV1HIP_RANGE_PRIO=3" ;;
    w0) E="FFV1HIP_WALK_PRIO=0" ;;
    w0r1) E="FFV1HIP_WALK_PRIO=0 FFV1HIP_RANGE_PRIO=1" ;;
    w1r3) E="FFV1HIP_WALK_PRIO=1 FFV1HIP_RANGE_PRIO=3" ;;
    r3big) E="FFV1HIP_RANGE_PRIO=3 FFV1HIP_SYM_GRID=4096 FFV1HIP_BITS_GRID=2048 FFV1HIP_DSEG_GRID=4096" ;;
    w0r3) E="FFV1HIP_WALK_PRIO=0 FFV1HIP_RANGE_PRIO=3" ;;
  esac
  env $E FFV1HIP_WALKTRACE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 20 --gops 20 > $O/b_$v.json 2> $O/b_$v.err || exit 4
done
echo done
