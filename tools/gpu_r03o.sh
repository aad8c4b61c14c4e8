set -u
mkdir -p gpurun_out/r03o
export TMPDIR=/tmp
bash tools/gpu_tests.sh r03o &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r03o/tl -o run -- python3 tools/build_timeline.py > gpurun_out/r03o/tl.log 2>&1 &&
python3 tools/build_timeline.py --analyze gpurun_out/r03o/tl > gpurun_out/r03o/timeline.txt 2>&1 &&
timeout -k 10 300 python3 tools/build_timeline.py --reps 9 > gpurun_out/r03o/noprof.log 2>&1 &&
timeout -k 10 600 python3 -u bench.py --no-cpu > gpurun_out/r03o/bench.json 2> gpurun_out/r03o/bench.err
