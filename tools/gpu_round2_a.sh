set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread -k "avcodec or config3" > gpurun_out/t_enc2.log 2>&1
timeout -k 10 240 python bench.py --steps 10 > gpurun_out/bench1.log 2>&1
FFV1_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 4 --gops 6 --no-cpu-baseline > gpurun_out/bench2.log 2>&1
timeout -k 10 300 python tools/bench_host.py 21 2 gpurun_out/host_rates.json > gpurun_out/host.log 2>&1
