#!/bin/bash
# Kernel timeline of a short bench run (rocprofv3 --kernel-trace only):
#   usage: gpu_timeline.sh TAG [bench args]; output gpurun_out/tl_<tag>/
set -o pipefail
TAG=${1:-tl}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tl_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
shift || true
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --warmup 1 --no-cpu-baseline --no-decode-check "$@" > $O/kt.log 2>&1 || exit 1
f=$(find $O/kt -name "*kernel_trace.csv" | head -1)
cp "$f" $O/kernel_trace.csv
echo done
