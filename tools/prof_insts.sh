#!/bin/bash
# Instruction mix per kernel of the bench workload (run under gpurun): two
# separate --pmc passes (SQ block: at most 8 counters a pass), never with
# trace options.  Usage: tools/prof_insts.sh TAG [bench.py args]
set -o pipefail
TAG=${1:-insts}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
shift || true
BENCH="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-decode-check $*"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $O/p1 -o p1 --output-format csv -- python3 $BENCH > $O/p1.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH -d $O/p2 -o p2 --output-format csv -- python3 $BENCH > $O/p2.log 2>&1 || exit 2
echo done
