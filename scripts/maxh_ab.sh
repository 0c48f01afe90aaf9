#!/bin/bash
# A/B of the history-space threshold (FRECSYS_DUAL_MAX_H) on one workload:
# alternating bench lines, ms per epoch and the two half-steps' times.
# Usage: maxh_ab.sh <outdir under gpurun_out> <workload> <steps> <reps> <max_h...>
#   (max_h "def" = the library default)
set -o pipefail
OUT=gpurun_out/$1; WL=$2; STEPS=$3; REPS=$4; shift 4
mkdir -p $OUT
for rep in $(seq 1 $REPS); do
  for m in "$@"; do
    if [ $m = def ]; then E=FRECSYS_NONE=0; else E=FRECSYS_DUAL_MAX_H=$m; fi
    env $E timeout -k 10 300 python bench.py --allow-env --workload $WL --extras= --cpu-seconds 0 --steps $STEPS --warmup 1 --quiet > $OUT/${WL}_${m}_$rep.json 2> $OUT/${WL}_${m}_$rep.err || { echo "$m failed"; tail -5 $OUT/${WL}_${m}_$rep.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['kernel_ms_per_epoch'];print(sys.argv[2], round(d['ms_per_step'],2), 'user', round(k['solve_user'],2), 'item', round(k['solve_item'],2), 'reruns', d['hspace_reruns'])" $OUT/${WL}_${m}_$rep.json ${WL}_${m}_$rep
  done
done
