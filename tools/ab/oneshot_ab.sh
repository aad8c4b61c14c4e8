set -u
for r in 1 2 3; do
  for lib in tools/ab/libshadow_gpu_prev.so shadow_amd/libshadow_gpu.so; do
    echo -n "$lib "; SHADOW_GPU_LIB=$PWD/$lib timeout -k 10 120 python3 tools/oneshot_parts.py 10000 || exit 1
  done
done
