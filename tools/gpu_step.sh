set -u
O=gpurun_out/r8h; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_routing_gpu.py tests/test_routing_fuzz_gpu.py -x -q --timeout 300 --timeout-method thread -k "bucket or band_degree" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 600 python3 -u -m pytest tests/test_c5_gpu.py -x -q --timeout 500 --timeout-method thread > $O/t5.log 2>&1 || { tail -30 $O/t5.log; exit 1; }
tail -1 $O/t5.log
timeout -k 10 600 python3 -u bench.py --config c5 --no-cpu --no-gml --no-c2 --steps 3 --warmup 1 --rank-blocks "" > $O/bench_c5.json 2> $O/bench_c5.err || { tail -5 $O/bench_c5.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open('$O/bench_c5.json').read().strip().splitlines()[-1]); print(d['value'], d['apsp_detail'].get('same_graph_rebuild_ms'), d['roofline'].get('avg_launch_ms'))"
