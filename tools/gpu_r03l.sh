set -u
mkdir -p gpurun_out/r03l
timeout -k 10 300 python3 -u tools/sssp_ab.py --reps 9 "SG_SSSP_PREFILTER=0" "SG_SSSP_PREFILTER=1" "SG_SSSP_PREFILTER=0" "SG_SSSP_PREFILTER=1" "SG_SSSP_PREFILTER=1,SG_SSSP_LANE_ARCS=16" > gpurun_out/r03l/ab_prefilter.txt 2>&1
