set -e
mkdir -p gpurun_out
FFV1HIP_SERIAL=1 FFV1HIP_WALKDBG=1 FFV1HIP_CODEDBG=1 timeout -k 10 240 python bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline --no-decode-check > gpurun_out/wdbg4.log 2>&1
