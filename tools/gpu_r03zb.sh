set -u
mkdir -p gpurun_out/r03zb
bash tools/gpu_tests.sh r03zb -k "deliver or bucket or dist or rccl or c5" &&
timeout -k 10 300 python3 -u bench.py --no-cpu --no-compare --no-gml --no-c2 --steps 5 --warmup 2 > gpurun_out/r03zb/bench.json 2> gpurun_out/r03zb/bench.err
