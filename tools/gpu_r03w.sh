set -u
mkdir -p gpurun_out/r03w
timeout -k 10 300 python3 -u tools/sssp_ab.py --reps 7 "SG_SSSP_SEEDS=1" "SG_APSP_DELTA=200000000" "SG_APSP_DELTA=100000000" "SG_APSP_DELTA=400000000" "SG_SSSP_CLAIM=32" "SG_SSSP_SEEDS=1" > gpurun_out/r03w/ab.txt 2>&1
