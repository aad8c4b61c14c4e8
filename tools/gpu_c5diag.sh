# C5 lane-kernel block timing (SG_LANE_DIAG=1): bench.py --config c5 without the comparison legs
set -u
O=gpurun_out/${C5DIAG_OUT:-r04za}; mkdir -p $O
export TMPDIR=/tmp
SG_LANE_DIAG=1 timeout -k 10 600 python3 -u bench.py --config c5 --no-cpu --no-gml --no-c2 --no-compare --steps 1 --warmup 0 --rank-blocks '' > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
grep "\[lane\]" $O/bench.err | sort | uniq -c | sort -rn | head -3 > /dev/null
for k in k_codel k_inbound k_outbound; do grep "\[lane\] $k" $O/bench.err | head -2; done
