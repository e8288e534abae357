#!/bin/bash
# tools/exp/build_variant.sh NAME KERNELS.hip [extra hipcc flags]: the library
# with another ffv1_kernels.hip into lib/exp/libNAME.so (A/B runs select it
# with FFV1HIP_LIB)
set -e
R=$(cd $(dirname $0)/../.. && pwd)
C=$R/ffmpeg-ffv1-p-frames_amd/csrc
mkdir -p $R/ffmpeg-ffv1-p-frames_amd/lib/exp
N=$1; K=$2; shift 2
cp $K /tmp/variant_kernels_$N.hip
cp $C/ffv1_internal.h /tmp/ffv1_internal.h
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-function -I $R/include -I $C "$@" \
  -o $R/ffmpeg-ffv1-p-frames_amd/lib/exp/lib$N.so /tmp/variant_kernels_$N.hip $C/ffv1_decode.hip $C/ffv1_host.cpp $C/ffv1_twopass.cpp
echo built lib/exp/lib$N.so
