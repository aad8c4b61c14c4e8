set -u
mkdir -p gpurun_out/r03i
timeout -k 10 600 python3 -u tools/apsp_variants.py --nodes 50000 --reps 1 --rounds 2 --variants "SG_APSP_GROUP_MB=4096;SG_APSP_GROUP_MB=1024;SG_APSP_GROUP_MB=512;SG_APSP_GROUP_MB=256;SG_APSP_B=32;SG_APSP_GROUP_MB=8192" > gpurun_out/r03i/c5_slab_ab.txt 2>&1
