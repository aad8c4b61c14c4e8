set -u
mkdir -p gpurun_out/r03d
bash tools/gpu_tests.sh r03d &&
timeout -k 10 600 python3 -u bench.py > gpurun_out/r03d/bench.json 2> gpurun_out/r03d/bench.err
