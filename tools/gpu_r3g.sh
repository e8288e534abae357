#!/bin/bash
# Round 3: host-frame pipeline and alpha / v4 parity, the PCIe-inclusive
# rates, then the c3 schedule: default vs walk / range waves owning their
# SIMD (FFV1HIP_WALK_FAT / FFV1HIP_RANGE_FAT), with kernel timelines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "encode2 or host_encode or avcodec or never_truncates or overflow" > $O/parity.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_alpha.py tests/test_v4.py > $O/alpha.log 2>&1 || exit 2
FFV1HIP_WALK_FAT=1 FFV1HIP_RANGE_FAT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "split_walk or device_path or full_size" > $O/fat_parity.log 2>&1 || exit 3
for v in def walkfat rangefat both; do
  case $v in
    def) E="" ;;
    walkfat) E="FFV1HIP_WALK_FAT=1" ;;
    rangefat) E="FFV1HIP_RANGE_FAT=1" ;;
    both) E="FFV1HIP_WALK_FAT=1 FFV1HIP_RANGE_FAT=1" ;;
  esac
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 10 > $O/bench_$v.json 2> $O/bench_$v.err || exit 4
done
timeout -k 10 600 python tools/bench_host.py 21 10 $O/host_rates.json > $O/host.log 2>&1 || exit 5
bash tools/gpu_timeline.sh r3g_def --steps 6 || exit 6
FFV1HIP_WALK_FAT=1 FFV1HIP_RANGE_FAT=1 bash tools/gpu_timeline.sh r3g_both --steps 6 || exit 7
echo done
