set -u
mkdir -p gpurun_out/r03zc
timeout -k 10 300 python3 -u tools/sssp_ab.py --reps 9 "SG_SSSP_PHASES=3" "SG_SSSP_PHASES=2" "SG_SSSP_PHASES=4" "SG_SSSP_BOUNDS=3" "SG_SSSP_PHASES=3" > gpurun_out/r03zc/ab.txt 2>&1
