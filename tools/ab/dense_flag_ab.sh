# Dense searches writing every row's flag (no fill before a build) against the previous library
# (tools/ab/build_rev.sh HEAD prev): the whole -m gpu suite, then the C2 leg A/B.
set -u
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/dflag_tests.log 2>&1 || { tail -5 gpurun_out/dflag_tests.log; exit 1; }
tail -1 gpurun_out/dflag_tests.log
rm -f gpurun_out/ab_c2_dflag.txt
timeout -k 10 600 bash tools/ab/c2_lib_ab.sh gpurun_out/ab_c2_dflag.txt 4 tools/ab/libshadow_gpu_prev.so shadow_amd/libshadow_gpu.so > /dev/null 2>&1 || exit 1
