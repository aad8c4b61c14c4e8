set -u
mkdir -p gpurun_out/r03x
bash tools/gpu_tests.sh r03x &&
timeout -k 10 600 python3 -u bench.py > gpurun_out/r03x/bench.json 2> gpurun_out/r03x/bench.err &&
bash tools/profile_round.sh r03x
