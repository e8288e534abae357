#!/bin/bash
# Round 3, final library: the side grids once more (c3).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3ai
mkdir -p $O
for v in base s2 s6 d2 b4; do
  case $v in
    base) E="" ;;
    s2) E="FFV1HIP_SYM_GRID=2048" ;;
    s6) E="FFV1HIP_SYM_GRID=6144" ;;
    d2) E="FFV1HIP_DSEG_GRID=2048" ;;
    b4) E="FFV1HIP_BITS_GRID=4096" ;;
  esac
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 20 > $O/b_$v.json 2> $O/b_$v.err || exit 1
done
echo done
