# the default bench line twice (box check of the one-shot value)
set -u
O=gpurun_out/${1:-bo}; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 400 python3 -u bench.py --no-cpu --no-gml --no-c2 > $O/b$i.json 2> $O/b$i.err || { tail -5 $O/b$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/b$i.json').read().strip().splitlines()[-1]); a=d['apsp_detail']; print('value', d['value'], 'rebuild', a['same_graph_rebuild_ms'], 'plan', a['plan_ms'])"
done
