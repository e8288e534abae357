#!/bin/bash
# Round 3: symbols with the quant tables in global memory (no LDS beside the
# walk): the schedule with and without the wait for part A; host rates with
# the copy-out breakdown.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3p
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "split_walk or full_size or batch or c3 or host_encode or encode2" > $O/parity.log 2>&1 || exit 1
for v in s4b1d4 s4b1d4z n4b1d3 n3b1d3 n6b2d3 n2b1d4; do
  case $v in
    s4b1d4) E="FFV1HIP_SYM_GRID=4096 FFV1HIP_BITS_GRID=1024 FFV1HIP_DSEG_GRID=4096" ;;
    s4b1d4z) E="FFV1HIP_SYM_GRID=4096 FFV1HIP_BITS_GRID=1024 FFV1HIP_DSEG_GRID=4096 FFV1HIP_SYM_DELAY_US=0" ;;
    n4b1d3) E="FFV1HIP_SYM_GRID=4096 FFV1HIP_BITS_GRID=1024 FFV1HIP_DSEG_GRID=3072 FFV1HIP_SYM_AFTER_A=0 FFV1HIP_SYM_DELAY_US=0" ;;
    n3b1d3) E="FFV1HIP_SYM_GRID=3072 FFV1HIP_BITS_GRID=1024 FFV1HIP_DSEG_GRID=3072 FFV1HIP_SYM_AFTER_A=0 FFV1HIP_SYM_DELAY_US=0" ;;
    n6b2d3) E="FFV1HIP_SYM_GRID=6144 FFV1HIP_BITS_GRID=2048 FFV1HIP_DSEG_GRID=3072 FFV1HIP_SYM_AFTER_A=0 FFV1HIP_SYM_DELAY_US=0" ;;
    n2b1d4) E="FFV1HIP_SYM_GRID=2048 FFV1HIP_BITS_GRID=1024 FFV1HIP_DSEG_GRID=4096 FFV1HIP_SYM_AFTER_A=0 FFV1HIP_SYM_DELAY_US=0" ;;
  esac
  env $E FFV1HIP_WALKTRACE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 10 > $O/b_$v.json 2> $O/b_$v.err || exit 4
done
FFV1HIP_SYM_GRID=4096 FFV1HIP_BITS_GRID=1024 FFV1HIP_DSEG_GRID=4096 FFV1HIP_WALKDBG=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 3 > $O/b_dbg.json 2> $O/b_dbg.err || exit 5
FFV1HIP_SYM_GRID=4096 FFV1HIP_BITS_GRID=1024 FFV1HIP_DSEG_GRID=4096 FFV1HIP_HOSTDBG=1 timeout -k 10 600 python tools/bench_host.py 21 10 $O/host_rates.json > $O/host.log 2>&1 || exit 3
echo done
