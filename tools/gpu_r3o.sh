#!/bin/bash
# Round 3: 8-byte walk records (the walk derives the slot codes per chunk):
# the GPU suite, then c3 with the bounded grids, the symbols after part A
# (default) or beside the whole walk (FFV1HIP_SYM_AFTER_A=0, small grid).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3o
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $O/gpu.log 2>&1 || exit 1
for v in s4b1d4 e1024 e768 e1024d50; do
  case $v in
    s4b1d4) E="FFV1HIP_SYM_GRID=4096 FFV1HIP_BITS_GRID=1024 FFV1HIP_DSEG_GRID=4096" ;;
    e1024) E="FFV1HIP_SYM_GRID=1024 FFV1HIP_BITS_GRID=1024 FFV1HIP_DSEG_GRID=4096 FFV1HIP_SYM_AFTER_A=0 FFV1HIP_SYM_DELAY_US=300" ;;
    e768) E="FFV1HIP_SYM_GRID=768 FFV1HIP_BITS_GRID=768 FFV1HIP_DSEG_GRID=4096 FFV1HIP_SYM_AFTER_A=0 FFV1HIP_SYM_DELAY_US=300" ;;
    e1024d50) E="FFV1HIP_SYM_GRID=1024 FFV1HIP_BITS_GRID=1024 FFV1HIP_DSEG_GRID=4096 FFV1HIP_SYM_AFTER_A=0 FFV1HIP_SYM_DELAY_US=50" ;;
  esac
  env $E FFV1HIP_WALKTRACE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 10 > $O/b_$v.json 2> $O/b_$v.err || exit 4
done
echo done
