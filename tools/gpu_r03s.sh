set -u
mkdir -p gpurun_out/r03s
timeout -k 10 600 python3 -u bench.py > gpurun_out/r03s/bench.json 2> gpurun_out/r03s/bench.err &&
bash tools/profile_round.sh r03s
