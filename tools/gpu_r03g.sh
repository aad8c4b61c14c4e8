set -u
mkdir -p gpurun_out/r03g
bash tools/gpu_tests.sh r03g -k "routing" &&
timeout -k 10 300 python3 -u tools/sssp_ab.py --reps 9 "SG_SSSP_LANDMARKS=0" "SG_SSSP_LANDMARKS=256" "SG_SSSP_LANDMARKS=128" "SG_SSSP_LANDMARKS=512" "SG_SSSP_LANDMARKS=0" "SG_SSSP_LANDMARKS=256,SG_SSSP_BOUNDS=3" > gpurun_out/r03g/ab_landmarks.txt 2>&1 &&
bash tools/gpu_r03f.sh
SG_LANE_DIAG=1 timeout -k 10 300 python3 -u bench.py --no-cpu --no-gml --no-c2 --no-compare --steps 2 --warmup 1 > gpurun_out/r03g/lane_diag.json 2> gpurun_out/r03g/lane_diag.err
