set -u
mkdir -p gpurun_out/r03zf
bash tools/gpu_tests.sh r03zf &&
timeout -k 10 600 python3 -u bench.py > gpurun_out/r03zf/bench.json 2> gpurun_out/r03zf/bench.err &&
bash tools/profile_round.sh r03zf
