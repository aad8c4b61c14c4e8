set -u
mkdir -p gpurun_out/r03m
bash tools/gpu_tests.sh r03m &&
timeout -k 10 600 python3 -u bench.py > gpurun_out/r03m/bench.json 2> gpurun_out/r03m/bench.err &&
bash tools/profile_round.sh r03m
