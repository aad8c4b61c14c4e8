set -u
O=gpurun_out/r6p; mkdir -p $O
B="SG_APSP_BUCKET=1"
timeout -k 10 900 python3 -u tools/apsp_ab.py --nodes 50000 --variants "$B;$B SG_BUCKET_DELTA=500000 SG_BUCKET_HASH=10;$B SG_BUCKET_DELTA=333333 SG_BUCKET_HASH=10;$B SG_BUCKET_DELTA=250000 SG_BUCKET_HASH=9;$B SG_BUCKET_DELTA=500000" --reps 1 --rounds 2 > $O/ab.log 2>&1; rc=$?; grep -E "median|round|identical" $O/ab.log; exit $rc
