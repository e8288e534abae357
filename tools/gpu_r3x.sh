#!/bin/bash
# Round 3: decision bits written by the walk (no ffv1_bits); dseg reading
# whole lines (128-decision blocks): its grid, its PMC FETCH_SIZE.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3x
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_fate.py tests/test_gpu_twopass.py tests/test_gpu_decoder.py > $O/parity.log 2>&1 || exit 1
for v in def kern d2k d8k; do
  case $v in
    def) E="" ;;
    kern) E="FFV1HIP_BITS_KERNEL=1" ;;
    d2k) E="FFV1HIP_DSEG_GRID=2048" ;;
    d8k) E="FFV1HIP_DSEG_GRID=8192" ;;
  esac
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 20 > $O/b_$v.json 2> $O/b_$v.err || exit 4
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in def; do
  case $v in
    def) E="" ;;
  esac
  env $E timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/$O/pmc_$v -o f --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-decode-check > $R/$O/pmc_$v.log 2>&1 || exit 5
done
echo done
