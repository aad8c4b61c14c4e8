set -u
mkdir -p gpurun_out/r03y
bash tools/gpu_tests.sh r03y &&
timeout -k 10 600 python3 -u bench.py > gpurun_out/r03y/bench.json 2> gpurun_out/r03y/bench.err &&
bash tools/profile_round.sh r03y
