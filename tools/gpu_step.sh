set -u
O=gpurun_out/r6r; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_inbound_gpu.py tests/test_codel_gpu.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 600 python3 -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); i=d['inbound']; print('inbound', i['ms_per_window'], i['roofline']['avg_launch_ms'], i['by_packet_id'])
print('delivery', d['delivery']['ms_per_round'] if 'delivery' in d else d.get('ms_per_step'))"
