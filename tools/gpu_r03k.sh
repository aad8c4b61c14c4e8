set -u
mkdir -p gpurun_out/r03k
bash tools/gpu_tests.sh r03k -k "team and (routing_gpu or fuzz)" &&
timeout -k 10 300 python3 -u tools/team_diag.py --nodes 50000 --reps 1 "SG_SSSP_TEAM=-1" "SG_SSSP_TEAM=8" > gpurun_out/r03k/team_diag3.txt 2>&1
