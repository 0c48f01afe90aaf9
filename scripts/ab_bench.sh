#!/bin/bash
# A/B of kernel variants selected by FRECSYS_DEBUG_SKIP masks: bench.py
# ms_per_step (+ the serialised per-kernel trace) per mask.
# Usage: ab_bench.sh <outdir> <mask> [<mask> ...]
set -o pipefail
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
  FRECSYS_DEBUG_SKIP=$m timeout -k 10 240 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/bench_$m.json 2> $OUT/bench_$m.err || exit 2
  FRECSYS_DEBUG_SKIP=$m FRECSYS_DUAL_SERIAL=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_$m -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 > $OUT/trace_$m.log 2>&1 || exit 3
done
echo ok
