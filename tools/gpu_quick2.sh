set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_fate.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/tq.log 2>&1
timeout -k 10 240 python bench.py --steps 20 --no-cpu-baseline > gpurun_out/bq.log 2>&1
timeout -k 10 240 python bench.py --steps 6 --config c4 --no-cpu-baseline > gpurun_out/bq4.log 2>&1
