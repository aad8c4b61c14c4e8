set -u
mkdir -p gpurun_out/r03zd
timeout -k 10 600 python3 -u bench.py --config c5 --no-cpu --no-compare --steps 2 --warmup 1 > gpurun_out/r03zd/bench_c5.json 2> gpurun_out/r03zd/bench_c5.err
