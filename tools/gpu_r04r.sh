set -u
O=gpurun_out/r04r; mkdir -p $O
export TMPDIR=/tmp
for T in 2560 1900 1280 900; do
  for TL in "" 0; do
    if [ -n "$TL" ]; then export SG_BUCKET_TWO_LEVEL=$TL; else unset SG_BUCKET_TWO_LEVEL; fi
    SG_SB_TARGET=$T timeout -k 10 200 python3 tools/round_c5.py --rounds 30 --nodes 10000 --hosts 100000 --packets 1000000 > $O/c4_$T$TL.log 2>&1 || exit 1
    echo "C4 target=$T twolevel=${TL:-auto}: $(tail -20 $O/c4_$T$TL.log | awk '{print $3}' | sort -n | head -10 | tail -1) ms (10th best of 20)"
  done
done
unset SG_BUCKET_TWO_LEVEL
for T in 2560 2000 3000; do
  SG_SB_TARGET=$T timeout -k 10 200 python3 tools/round_c5.py --rounds 10 > $O/c5_$T.log 2>&1 || exit 1
  echo "C5 target=$T: $(tail -6 $O/c5_$T.log | awk '{print $3}' | sort -n | head -3 | tail -1) ms (3rd best of 6)"
done
