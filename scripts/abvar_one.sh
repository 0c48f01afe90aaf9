#!/bin/bash
# A/B library that differs from the tree's in ONE source file: that file
# recompiled with extra defines, linked with the tree's other objects
# (safer2-recommender_amd/build/*.o, `make lib` first).
# Usage: abvar_one.sh <name> <source.hip> <defines...>
#   -> ab/libfrecsys_hip_<name>.so   (scripts/ab_compare.sh / msd_ab.sh swap it in)
set -e
NAME=$1 SRC=$2
shift 2
OBJ=safer2-recommender_amd/build
mkdir -p ab/obj/$NAME
BASE=$(basename $SRC .hip)
EXTRA=""
[ "$BASE" = wide_syrk ] && EXTRA=-fno-slp-vectorize
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result $EXTRA "$@" \
  -c $SRC -o ab/obj/$NAME/$BASE.o
OBJS=$(ls $OBJ/*.o | grep -v "/$BASE.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ab/libfrecsys_hip_$NAME.so $OBJS ab/obj/$NAME/$BASE.o -lrccl
echo ab/libfrecsys_hip_$NAME.so
