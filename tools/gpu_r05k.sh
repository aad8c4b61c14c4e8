# host API timing of the C4 round (hip runtime trace + kernel trace of tools/round_c4.py)
set -u
export TMPDIR=/tmp
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 150 rocprofv3 --hip-runtime-trace --kernel-trace --output-format csv -d $O/t -o run -- python3 tools/round_c4.py "" > $O/t.log 2>&1 || { tail -5 $O/t.log; exit 1; }
ls -R $O/t | head -20
