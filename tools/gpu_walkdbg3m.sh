set -e
mkdir -p gpurun_out
FFV1HIP_FORCE_MULTI=1 FFV1HIP_SERIAL=1 FFV1HIP_WALKDBG=1 timeout -k 10 240 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-decode-check > gpurun_out/wdbg3m.log 2>&1
