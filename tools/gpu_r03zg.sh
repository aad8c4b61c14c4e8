set -u
mkdir -p gpurun_out/r03zg
timeout -k 10 300 python3 -u tools/sssp_ab.py --reps 9 "SG_SSSP_LANE_ARCS=8" "SG_SSSP_LANE_ARCS=16" "SG_SSSP_LANE_DEG=12" "SG_SSSP_LANE_DEG=24" "SG_SSSP_LANE_ARCS=8" > gpurun_out/r03zg/ab.txt 2>&1
