#!/bin/bash
# SQ counters of the pipeline kernels on a short serial bench run (one pass
# per counter group; never combined with traces).  Output: gpurun_out/pmc_<tag>/
set -o pipefail
TAG=${1:-walk}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export FFV1HIP_DEBUG=serial
BENCH="$R/bench.py --steps 1 --warmup 0 --gops ${GOPS:-2} --no-cpu-baseline"
timeout -k 10 300 python3 $BENCH > $O/plain.json 2> $O/plain.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $BENCH > $O/kt.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_WAIT_ANY -d $O/p1 -o p1 --output-format csv -- python3 $BENCH > $O/p1.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/p2 -o p2 --output-format csv -- python3 $BENCH > $O/p2.log 2>&1 || exit 4
echo done
