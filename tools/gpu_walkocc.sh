set -e
mkdir -p gpurun_out
for pad in 0 20000 60000; do
echo "pad $pad" >> gpurun_out/wocc.log
FFV1HIP_WALK_LDS_PAD=$pad FFV1HIP_SERIAL=1 FFV1HIP_WALKDBG=1 timeout -k 10 240 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-decode-check >> gpurun_out/wocc.log 2>&1
done
