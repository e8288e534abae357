#!/bin/bash
# SQ counters of the chained range coder on one bgr0 case (tools/bench_chained.py),
# two --pmc passes, no traces (run under gpurun); summarise with
#   python3 tools/sq_summary.py gpurun_out/sq_chain
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/sq_chain
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/tools/bench_chained.py $O/rates.json 1 bgr0_1080p_s24_g12"
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $O/p1 -o p1 --output-format csv -- python3 $B > $O/p1.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH -d $O/p2 -o p2 --output-format csv -- python3 $B > $O/p2.log 2>&1 || exit 2
echo done
