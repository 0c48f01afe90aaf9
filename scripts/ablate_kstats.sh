#!/bin/bash
# Phase ablations of the ablation build (FRECSYS_DEBUG_SKIP masks, timing only:
# the results are wrong), streams serialised: rocprofv3 kernel stats per mask.
# Usage: ablate_kstats.sh <outdir under gpurun_out> <workload> <mask...>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; W=$2; shift 2
mkdir -p $OUT
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
cp $LIB $OUT/tree.so.bak
trap 'cp $OUT/tree.so.bak $LIB; rm -f $OUT/tree.so.bak' EXIT
cp ab/libfrecsys_hip_ablation.so $LIB
S=3; [ $W = ials_ml20m_d256 ] && S=8
for m in "$@"; do
  FRECSYS_DEBUG_SKIP=$m FRECSYS_DUAL_SERIAL=1 timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/t_$m -o run --output-format csv -- python3 bench.py --allow-env --workload $W --extras= --cpu-seconds 0 --steps $S --warmup 1 --quiet > $OUT/t_$m.log 2>&1 || { echo "mask $m failed"; tail -3 $OUT/t_$m.log; exit 1; }
  python3 scripts/kstats.py $OUT/t_$m/run_kernel_stats.csv $((S + 1)) 30 > $OUT/kstats_$m.txt
  rm -f $OUT/t_$m/*kernel_trace.csv
  echo "== mask $m"; grep -E "dual_|solve_tiled|total" $OUT/kstats_$m.txt
done
