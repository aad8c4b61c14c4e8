set -u
mkdir -p gpurun_out/r03za
SG_NET_LDS=1 bash tools/gpu_tests.sh r03za -k "routing or c2 or capi or gml or dist" &&
timeout -k 10 300 python3 -u bench.py --no-cpu --no-compare --steps 3 --warmup 1 > gpurun_out/r03za/bench.json 2> gpurun_out/r03za/bench.err &&
SG_NET_LDS=1 timeout -k 10 300 python3 -u bench.py --no-cpu --no-compare --steps 3 --warmup 1 > gpurun_out/r03za/bench_lds.json 2>> gpurun_out/r03za/bench.err
