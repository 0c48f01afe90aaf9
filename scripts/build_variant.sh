#!/bin/bash
# Build a variant of libfrecsys_hip.so with extra -D flags on one source
# (the other objects from the in-tree build): ab/v/<name>.so
# Usage: build_variant.sh <name> <source.hip> [-DFLAG=...]
set -e
cd "$(dirname "$0")/.."
NAME=$1; SRC=$2; shift 2
mkdir -p ab/obj ab/v
B=$(basename $SRC .hip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result "$@" -c safer2-recommender_amd/csrc/$SRC -o ab/obj/${B}_$NAME.o
OBJS=$(ls safer2-recommender_amd/build/*.o | grep -v "/$B.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ab/v/$NAME.so $OBJS ab/obj/${B}_$NAME.o -lrccl
echo ab/v/$NAME.so
