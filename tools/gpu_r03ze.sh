set -u
mkdir -p gpurun_out/r03ze
SG_BENCH_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu > gpurun_out/r03ze/bench_n2.json 2> gpurun_out/r03ze/bench_n2.err
