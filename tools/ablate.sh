#!/bin/bash
# Timing-only ablation builds of ffv1_code (outputs are not valid bitstreams).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
for A in 1 2 4 7; do
  mkdir -p $R/gpurun_out/ablate$A
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DFFV1_ABLATE=$A -I $R/include \
    -o $R/ffmpeg-ffv1-p-frames_amd/lib/libffv1hip_ablate$A.so \
    $R/ffmpeg-ffv1-p-frames_amd/csrc/ffv1_kernels.hip $R/ffmpeg-ffv1-p-frames_amd/csrc/ffv1_host.cpp
done
