#!/bin/bash
# Serialised kernel trace of bench.py under FRECSYS_DEBUG_SKIP ablation masks
# (results are garbage under a mask; only the kernel times are read).
# Usage: ablate_trace.sh <outdir> <mask> [<mask> ...]
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
# the masks exist only in the ablation build (make ablation); swap it in
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
cp $LIB /tmp/libfrecsys_hip.release.so && cp ab/libfrecsys_hip_ablation.so $LIB || exit 9
trap 'cp /tmp/libfrecsys_hip.release.so $LIB' EXIT
OUT=gpurun_out/$1
shift
mkdir -p $OUT
for m in "$@"; do
  FRECSYS_DEBUG_SKIP=$m FRECSYS_DUAL_SERIAL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace_$m -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 > $OUT/trace_$m.log 2>&1
done
echo done
