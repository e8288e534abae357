#!/bin/bash
# Kernel times of the decoder (rocprofv3 stats over a short c3 bench with its decode self-check).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/decprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 2 > $O/kt.log 2>&1 || exit 1
timeout -k 10 400 env FFV1HIP_DEC_SWAP=0 rocprofv3 --kernel-trace --stats -d $O/kt0 -o kt --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 2 > $O/kt0.log 2>&1 || exit 2
echo done
