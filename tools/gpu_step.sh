set -u
O=gpurun_out/r8z; mkdir -p $O
SG_NET_TRACE=1 timeout -k 10 200 python3 -u tools/oneshot_parts.py 1250 > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
grep -v amdgpu $O/p.log | tail -6
