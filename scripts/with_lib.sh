#!/bin/bash
# Run a command with ab/libfrecsys_hip_<name>.so swapped in for the tree's
# library (restored on exit).  Usage: with_lib.sh <name> <command...>
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
cp $LIB /tmp/tree_lib.so.bak
trap 'cp /tmp/tree_lib.so.bak $LIB' EXIT
cp ab/libfrecsys_hip_$1.so $LIB
shift
"$@"
