#!/bin/bash
# Round 3: bounded grids for the kernels beside the states walk (symbols,
# bits, dseg): parity with small caps (the blocks stride over the items),
# then a c3 sweep of the caps with the walk's per-wave trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3m
mkdir -p $O
FFV1HIP_SYM_GRID=300 FFV1HIP_BITS_GRID=100 FFV1HIP_DSEG_GRID=77 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "split_walk or full_size or device_path or batch or c3" > $O/parity.log 2>&1 || exit 1
for v in def d4 d2 s2b1d4 s4b1d4 s1b05d2; do
  case $v in
    def) E="" ;;
    d4) E="FFV1HIP_DSEG_GRID=4096" ;;
    d2) E="FFV1HIP_DSEG_GRID=2048" ;;
    s2b1d4) E="FFV1HIP_SYM_GRID=2048 FFV1HIP_BITS_GRID=1024 FFV1HIP_DSEG_GRID=4096" ;;
    s4b1d4) E="FFV1HIP_SYM_GRID=4096 FFV1HIP_BITS_GRID=1024 FFV1HIP_DSEG_GRID=4096" ;;
    s1b05d2) E="FFV1HIP_SYM_GRID=1024 FFV1HIP_BITS_GRID=512 FFV1HIP_DSEG_GRID=2048" ;;
  esac
  env $E FFV1HIP_WALKTRACE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 10 > $O/b_$v.json 2> $O/b_$v.err || exit 4
done
echo done
