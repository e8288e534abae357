cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pmc/kt -o kt --output-format csv -- python3 $R/tools/diag_one.py 3840 2160 64 1 12 > $R/gpurun_out/pmc/kt.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $R/gpurun_out/pmc/p1 -o p1 --output-format csv -- python3 $R/tools/diag_one.py 3840 2160 64 1 12 > $R/gpurun_out/pmc/p1.log 2>&1 || exit 2
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT -d $R/gpurun_out/pmc/p2 -o p2 --output-format csv -- python3 $R/tools/diag_one.py 3840 2160 64 1 12 > $R/gpurun_out/pmc/p2.log 2>&1 || exit 3
echo done
