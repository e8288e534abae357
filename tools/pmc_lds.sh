#!/bin/bash
# LDS counters of the walk, kernels one at a time (serial): bank conflicts,
# LDS-array cycles and LDS waits per launch (one rocprofv3 --pmc pass).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_lds
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export FFV1HIP_DEBUG=serial
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/p -o p --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-decode-check > $O/p.log 2>&1
