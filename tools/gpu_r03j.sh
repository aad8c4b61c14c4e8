set -u
mkdir -p gpurun_out/r03j
bash tools/gpu_tests.sh r03j -k "team and (routing_gpu or fuzz)" &&
timeout -k 10 300 python3 -u -m pytest tests/test_c5_gpu.py -x -v --timeout 240 -k table > gpurun_out/r03j/c5_table.log 2>&1 &&
timeout -k 10 600 python3 -u tools/apsp_variants.py --nodes 50000 --reps 1 --rounds 2 --variants "SG_SSSP_TEAM=-1;SG_APSP_LDS=0;SG_APSP_LDS=0 SG_APSP_GROUP_MB=1024;SG_APSP_LDS=0 SG_APSP_B=32" > gpurun_out/r03j/c5_ab.txt 2>&1
