set -u
mkdir -p gpurun_out/r03h
SG_LANE_HOSTS=32 bash tools/gpu_tests.sh r03h -k "codel or inbound or outbound" &&
SG_LANE_DIAG=1 SG_LANE_HOSTS=64 timeout -k 10 300 python3 -u bench.py --no-cpu --no-gml --no-c2 --no-compare --steps 2 --warmup 1 > gpurun_out/r03h/lane64.json 2> gpurun_out/r03h/lane64.err &&
SG_LANE_DIAG=1 SG_LANE_HOSTS=32 timeout -k 10 300 python3 -u bench.py --no-cpu --no-gml --no-c2 --no-compare --steps 2 --warmup 1 > gpurun_out/r03h/lane32.json 2> gpurun_out/r03h/lane32.err &&
SG_LANE_HOSTS=64 timeout -k 10 300 python3 -u bench.py --no-cpu --no-gml --no-c2 --no-compare --steps 5 --warmup 2 > gpurun_out/r03h/b64.json 2> gpurun_out/r03h/b64.err &&
SG_LANE_HOSTS=32 timeout -k 10 300 python3 -u bench.py --no-cpu --no-gml --no-c2 --no-compare --steps 5 --warmup 2 > gpurun_out/r03h/b32.json 2> gpurun_out/r03h/b32.err
