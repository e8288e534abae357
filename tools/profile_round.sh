#!/bin/bash
# Round profile of the bench workload on one MI355X (run under gpurun):
#   usage: profile_round.sh TAG [extra bench.py args, e.g. --config c4]
#   1. rocprofv3 --kernel-trace --stats of bench.py (per-kernel durations)
#   2. PMC FETCH_SIZE pass, 3. PMC WRITE_SIZE pass (separate passes: they
#      do not fit one pass; never combined with sys/runtime traces)
# Outputs under gpurun_out/prof_<tag>/; summarise with tools/pmc_summary.py.
set -o pipefail
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
shift || true
BENCH="$R/bench.py --warmup 1 --no-cpu-baseline $*"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $BENCH > $O/kt.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- python3 $BENCH > $O/fetch.log 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- python3 $BENCH > $O/write.log 2>&1 || exit 3
echo done
