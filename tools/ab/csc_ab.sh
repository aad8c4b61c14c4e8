# The lazy in-arc CSC (upload writes the out-arcs only) against the previous library
# (tools/ab/build_rev.sh HEAD prev): the whole -m gpu suite, upload kernels under the kernel
# trace (C3 block one-shots), the C2 one-shot A/B, then the C3 one-shot A/B.
set -u
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/csc_tests.log 2>&1 || { tail -5 gpurun_out/csc_tests.log; exit 1; }
tail -1 gpurun_out/csc_tests.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/csc_prof -o run -- python3 tools/oneshot_parts.py 1250 > /dev/null 2>&1 || exit 1
rm -f gpurun_out/ab_c2_csc.txt
timeout -k 10 600 bash tools/ab/c2_lib_ab.sh gpurun_out/ab_c2_csc.txt 3 tools/ab/libshadow_gpu_prev.so shadow_amd/libshadow_gpu.so > /dev/null 2>&1 || exit 1
timeout -k 10 500 bash tools/ab/oneshot_lib_ab.sh > gpurun_out/ab_csc.txt 2>&1 || exit 1
