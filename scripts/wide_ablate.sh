#!/bin/bash
# Ablation of the wide d-space kernels on one bench workload: the serialised
# kernel stats with FRECSYS_DEBUG_SKIP masks (ablation build swapped in;
# wide_syrk2: 1 = no MFMAs, 32 = no row gathers).
# Usage: wide_ablate.sh <outdir> <workload> <mask> [<mask> ...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
cp $LIB /tmp/libfrecsys_hip.release.so && cp ab/libfrecsys_hip_ablation.so $LIB || exit 9
trap 'cp /tmp/libfrecsys_hip.release.so $LIB' EXIT
OUT=gpurun_out/$1
W=$2
shift 2
mkdir -p $OUT
for m in "$@"; do
  FRECSYS_DEBUG_SKIP=$m FRECSYS_DUAL_SERIAL=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_$m -o run --output-format csv -- python3 bench.py --workload $W --extras= --allow-env --steps 1 --warmup 0 --cpu-seconds 0 --quiet > $OUT/trace_$m.log 2>&1 || { echo "mask $m failed"; tail -5 $OUT/trace_$m.log; exit 3; }
  echo "== mask $m"
  python3 scripts/kstats.py $OUT/trace_$m/run_kernel_stats.csv 1 | grep -E "wide_syrk2|wide_chol|total"
done
