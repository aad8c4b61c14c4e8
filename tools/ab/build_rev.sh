#!/bin/bash
# Build the library of a committed revision as tools/ab/libshadow_gpu_<name>.so (timing A/B only;
# load it with SHADOW_GPU_LIB=...).  usage: bash tools/ab/build_rev.sh REV NAME
set -e
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
SRC=/tmp/sg_rev_$NAME; rm -rf $SRC; mkdir -p $SRC
git -C $ROOT archive $REV shadow_amd/csrc include | tar -x -C $SRC
make -s -j8 -C $SRC/shadow_amd/csrc OUT=$ROOT/tools/ab/libshadow_gpu_$NAME.so OBJDIR=$SRC/obj
echo built tools/ab/libshadow_gpu_$NAME.so
