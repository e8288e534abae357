#!/bin/bash
# Round 3: host path with packets packed on the device (one D2H), then the
# c3 schedule: default, one records set, and R CUs reserved for the next
# batch's symbols / bits (FFV1HIP_RESERVE_CUS) with the walk in one launch.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3l
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "host_encode or encode2 or avcodec" > $O/parity.log 2>&1 || exit 1
FFV1HIP_RESERVE_CUS=32 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "split_walk or full_size or device_path or batch" > $O/parity_res.log 2>&1 || exit 2
FFV1HIP_HOSTDBG=1 timeout -k 10 600 python tools/bench_host.py 21 10 $O/host_rates.json > $O/host.log 2>&1 || exit 3
for v in def rec1 r16 r32 r48; do
  case $v in
    def) E="" ;;
    rec1) E="FFV1HIP_RECSETS=1" ;;
    r16) E="FFV1HIP_RESERVE_CUS=16" ;;
    r32) E="FFV1HIP_RESERVE_CUS=32" ;;
    r48) E="FFV1HIP_RESERVE_CUS=48" ;;
  esac
  env $E FFV1HIP_WALKTRACE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 10 > $O/b_$v.json 2> $O/b_$v.err || exit 4
done
echo done
