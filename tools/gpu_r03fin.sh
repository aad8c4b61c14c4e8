set -u
mkdir -p gpurun_out/r03fin
bash tools/gpu_tests.sh r03fin &&
timeout -k 10 600 python3 -u bench.py > gpurun_out/r03fin/bench.json 2> gpurun_out/r03fin/bench.err &&
bash tools/profile_round.sh r03fin
