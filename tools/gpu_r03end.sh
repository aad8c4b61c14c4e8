set -u
mkdir -p gpurun_out/r03end
bash tools/gpu_tests.sh r03end &&
timeout -k 10 600 python3 -u bench.py > gpurun_out/r03end/bench.json 2> gpurun_out/r03end/bench.err
