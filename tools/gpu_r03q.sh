set -u
mkdir -p gpurun_out/r03q
export TMPDIR=/tmp
bash tools/gpu_tests.sh r03q -k "routing or capi or gml" &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r03q/tl -o run -- python3 tools/build_timeline.py > gpurun_out/r03q/tl.log 2>&1 &&
python3 tools/build_timeline.py --analyze gpurun_out/r03q/tl > gpurun_out/r03q/timeline.txt 2>&1 &&
timeout -k 10 300 python3 tools/build_timeline.py --reps 9 > gpurun_out/r03q/noprof.log 2>&1
