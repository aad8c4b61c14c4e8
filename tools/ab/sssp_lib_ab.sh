# Interleaved A/B of the previous library (tools/ab/build_rev.sh HEAD prev) against the tree's,
# one-shot C3 builds: the whole table and an 8-way row block (tools/oneshot_parts.py).
set -u
for rows in 10000 1250; do
  for r in 1 2 3; do
    for lib in tools/ab/libshadow_gpu_prev.so shadow_amd/libshadow_gpu.so; do
      echo -n "$rows $lib "; SHADOW_GPU_LIB=$PWD/$lib timeout -k 10 120 python3 tools/oneshot_parts.py $rows || exit 1
    done
  done
done
