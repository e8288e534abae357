#!/bin/bash
# Round 3: bounded grids beside the walk; the symbols of batch k+1 also
# beside part A of batch k's walk (FFV1HIP_SYM_AFTER_A=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3n
mkdir -p $O
for v in s4b1d4 s4b1d4n s8b2d4n s2b1d4n s6b1d4 s4b1d6 s3b1d3n; do
  case $v in
    s4b1d4) E="FFV1HIP_SYM_GRID=4096 FFV1HIP_BITS_GRID=1024 FFV1HIP_DSEG_GRID=4096" ;;
    s4b1d4n) E="FFV1HIP_SYM_GRID=4096 FFV1HIP_BITS_GRID=1024 FFV1HIP_DSEG_GRID=4096 FFV1HIP_SYM_AFTER_A=0" ;;
    s8b2d4n) E="FFV1HIP_SYM_GRID=8192 FFV1HIP_BITS_GRID=2048 FFV1HIP_DSEG_GRID=4096 FFV1HIP_SYM_AFTER_A=0" ;;
    s2b1d4n) E="FFV1HIP_SYM_GRID=2048 FFV1HIP_BITS_GRID=1024 FFV1HIP_DSEG_GRID=4096 FFV1HIP_SYM_AFTER_A=0" ;;
    s6b1d4) E="FFV1HIP_SYM_GRID=6144 FFV1HIP_BITS_GRID=1024 FFV1HIP_DSEG_GRID=4096" ;;
    s4b1d6) E="FFV1HIP_SYM_GRID=4096 FFV1HIP_BITS_GRID=1024 FFV1HIP_DSEG_GRID=6144" ;;
    s3b1d3n) E="FFV1HIP_SYM_GRID=3072 FFV1HIP_BITS_GRID=1024 FFV1HIP_DSEG_GRID=3072 FFV1HIP_SYM_AFTER_A=0" ;;
  esac
  env $E FFV1HIP_WALKTRACE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 10 > $O/b_$v.json 2> $O/b_$v.err || exit 4
done
echo done
