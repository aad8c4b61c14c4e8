#!/bin/bash
# Build an experiment library tools/ab/libshadow_gpu_<name>.so with extra -D flags (timing A/B only).
# usage: bash tools/ab/build_variant.sh NAME "-DSG_EXPERIMENT_X"
set -e
NAME=$1; DEFS=$2
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OBJ=/tmp/sg_ab_$NAME; rm -rf $OBJ; mkdir -p $OBJ
cd $ROOT/shadow_amd/csrc
pids=()
for f in $(ls *.hip | sed 's/\.hip$//'); do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-result --offload-arch=gfx950 -ffp-contract=off \
    -fno-fast-math -munsafe-fp-atomics $DEFS -c $f.hip -o $OBJ/$f.o &
  pids+=($!)
done
g++ -O3 -std=c++17 -fPIC -Wall -c sg_gml.cpp -o $OBJ/sg_gml.o
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined -o $ROOT/tools/ab/libshadow_gpu_$NAME.so $OBJ/*.o
echo built tools/ab/libshadow_gpu_$NAME.so
