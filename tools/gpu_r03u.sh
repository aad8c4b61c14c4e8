set -u
mkdir -p gpurun_out/r03u
for R in 0:5000 0:2500 0:1250; do
timeout -k 10 200 python3 -u tools/sssp_ab.py --reps 9 --rows $R "SG_SSSP_SEEDS=1" "SG_SSSP_SEEDS=2" "SG_SSSP_SEEDS=2,SG_SSSP_PHASES=2" "SG_SSSP_SEEDS=0" >> gpurun_out/r03u/rows.txt 2>&1 || exit 1
done
