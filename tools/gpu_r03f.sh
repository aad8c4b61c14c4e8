set -u
mkdir -p gpurun_out/r03f
export MASTER_ADDR=127.0.0.1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_PORT=29611
timeout -k 10 300 python3 -u tools/rccl_check.py > gpurun_out/r03f/rccl_check.json 2> gpurun_out/r03f/rccl_check.err &&
SG_BENCH_BACKEND=gloo timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --steps 3 --warmup 2 --no-cpu --no-codel --no-gml --no-c2 --no-compare > gpurun_out/r03f/bench_n2_gloo.json 2> gpurun_out/r03f/bench_n2_gloo.err
