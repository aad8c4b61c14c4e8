set -u
mkdir -p gpurun_out/r03n
export TMPDIR=/tmp
bash tools/gpu_tests.sh r03n -k "routing or c3 or dist or rccl" &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r03n/tl -o run -- python3 tools/build_timeline.py > gpurun_out/r03n/tl.log 2>&1 &&
python3 tools/build_timeline.py --analyze gpurun_out/r03n/tl > gpurun_out/r03n/timeline.txt 2>&1
