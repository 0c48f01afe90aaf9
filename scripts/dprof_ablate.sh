#!/bin/bash
# History-space phase profile (FRECSYS_DUAL_PROF) under debug-skip ablation masks.
# Usage: dprof_ablate.sh <mask> [<mask> ...]   (0 = no ablation)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
# the masks exist only in the ablation build (make ablation); swap it in
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
cp $LIB /tmp/libfrecsys_hip.release.so && cp ab/libfrecsys_hip_ablation.so $LIB || exit 9
trap 'cp /tmp/libfrecsys_hip.release.so $LIB' EXIT
mkdir -p gpurun_out/dpa
for m in "$@"; do
  FRECSYS_DEBUG_SKIP=$m FRECSYS_DUAL_PROF=1 FRECSYS_DUAL_SERIAL=1 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --cpu-seconds 0 > gpurun_out/dpa/m$m.log 2>&1 || exit 1
done
