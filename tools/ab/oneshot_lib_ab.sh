# Interleaved A/B of the previous library (tools/ab/build_rev.sh HEAD prev) against the tree's:
# one-shot C3 builds of an 8-way row block and the whole table (tools/oneshot_parts.py), and
# the upload kernels' average times under the kernel trace are taken separately.
set -u
for rows in 1250 10000; do
  for r in 1 2 3; do
    for lib in tools/ab/libshadow_gpu_prev.so shadow_amd/libshadow_gpu.so; do
      out=$(SHADOW_GPU_LIB=$PWD/$lib timeout -k 10 120 python3 tools/oneshot_parts.py $rows 2>/dev/null) || exit 1
      echo "$rows $lib $out"
    done
  done
done
