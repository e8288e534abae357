#!/bin/bash
# The coder's segment pass, three ways of storing its digits (builds in
# lib/exp/): serial (no overlap) and overlapped kernel times.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3c
mkdir -p $O
for v in 0 1 2; do
  FFV1HIP_LIB=ffmpeg-ffv1-p-frames_amd/lib/exp/libffv1hip_v$v.so FFV1HIP_SERIAL=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 5 > $O/serial_v$v.json 2> $O/serial_v$v.err || exit 1
  FFV1HIP_LIB=ffmpeg-ffv1-p-frames_amd/lib/exp/libffv1hip_v$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-decode-check --steps 8 > $O/over_v$v.json 2> $O/over_v$v.err || exit 2
done
echo done
