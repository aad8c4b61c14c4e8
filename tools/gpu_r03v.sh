set -u
mkdir -p gpurun_out/r03v
bash tools/gpu_tests.sh r03v -k "codel or inbound or outbound" &&
bash tools/lane_stats.sh r03v > gpurun_out/r03v/lane.txt 2>&1
