set -u
O=gpurun_out/r8t; mkdir -p $O
for i in 1 2; do
  timeout -k 10 400 python3 -u bench.py --no-cpu --no-gml --no-c2 > $O/b$i.json 2> $O/b$i.err || { tail -5 $O/b$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/b$i.json').read().strip().splitlines()[-1]); a=d['apsp_detail']; print('value', d['value'], 'rebuild', a['same_graph_rebuild_ms'], {k: v['max_ms'] for k, v in a['rank_block_ms'].items()})"
done
