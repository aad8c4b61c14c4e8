set -u
mkdir -p gpurun_out/r03r
bash tools/gpu_tests.sh r03r &&
timeout -k 10 200 python3 tools/build_timeline.py --reps 9 > gpurun_out/r03r/host2.log 2>&1
