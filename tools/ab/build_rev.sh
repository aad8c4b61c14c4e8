#!/bin/bash
# Build the library of a committed revision as tools/ab/libshadow_gpu_<name>.so (timing A/B only).
# usage: bash tools/ab/build_rev.sh REV NAME
set -e
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
SRC=/tmp/sg_rev_$NAME; rm -rf $SRC; mkdir -p $SRC
git -C $ROOT archive $REV shadow_amd/csrc include | tar -x -C $SRC
cd $SRC/shadow_amd/csrc
pids=()
for f in sg_context sg_routing sg_deliver sg_codel; do
  [ -f $f.hip ] || continue
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-result --offload-arch=gfx950 -ffp-contract=off \
    -fno-fast-math -munsafe-fp-atomics -c $f.hip -o $f.o &
  pids+=($!)
done
g++ -O3 -std=c++17 -fPIC -Wall -c sg_gml.cpp -o sg_gml.o
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined -o $ROOT/tools/ab/libshadow_gpu_$NAME.so *.o
echo built tools/ab/libshadow_gpu_$NAME.so
