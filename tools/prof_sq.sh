#!/bin/bash
# SQ counters per kernel of the bench workload with every kernel alone
# (FFV1HIP_DEBUG=serial): wave cycles split into waiting (s_waitcnt),
# issue stalls and issuing, and the instruction mix.  Run under gpurun:
#   tools/prof_sq.sh TAG [bench.py args]    -> gpurun_out/sq_TAG/{p1,p2}
# Summarise with tools/sq_summary.py gpurun_out/sq_TAG
set -o pipefail
TAG=${1:-x}
shift || true
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/sq_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export FFV1HIP_DEBUG=serial${FFV1HIP_DEBUG:+,$FFV1HIP_DEBUG}
B="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-decode-check $*"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $O/p1 -o p1 --output-format csv -- python3 $B > $O/p1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT -d $O/p2 -o p2 --output-format csv -- python3 $B > $O/p2.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $B > $O/kt.log 2>&1 || exit 3
echo done
