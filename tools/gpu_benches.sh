# The round's bench lines: every BASELINE config on one GPU, D1 and D2 data.
set -e
mkdir -p gpurun_out/benches
timeout -k 10 300 python bench.py > gpurun_out/benches/c3.json 2> gpurun_out/benches/c3.err
timeout -k 10 300 python bench.py --data d2 --no-cpu-baseline > gpurun_out/benches/c3_d2.json 2> gpurun_out/benches/c3_d2.err
timeout -k 10 300 python bench.py --config c4 --steps 10 --no-cpu-baseline > gpurun_out/benches/c4.json 2> gpurun_out/benches/c4.err
timeout -k 10 300 python bench.py --config c2 --steps 10 --no-cpu-baseline > gpurun_out/benches/c2.json 2> gpurun_out/benches/c2.err
timeout -k 10 300 python bench.py --config c5 --steps 10 --no-cpu-baseline > gpurun_out/benches/c5.json 2> gpurun_out/benches/c5.err
