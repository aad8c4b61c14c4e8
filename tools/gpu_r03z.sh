set -u
mkdir -p gpurun_out/r03z
bash tools/gpu_tests.sh r03z -k "routing" &&
timeout -k 10 300 python3 -u tools/sssp_ab.py --reps 9 "SG_SSSP_SEEDS=1" "SG_SSSP_SEEDS=1" > gpurun_out/r03z/ab.txt 2>&1 &&
timeout -k 10 200 python3 tools/build_timeline.py --reps 9 > gpurun_out/r03z/host.log 2>&1
