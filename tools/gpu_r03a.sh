set -u
mkdir -p gpurun_out/r03a
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r03a/smoke.log 2>&1 &&
timeout -k 10 600 python3 -u bench.py > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err &&
bash tools/profile_round.sh r03a
