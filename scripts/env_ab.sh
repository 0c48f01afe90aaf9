#!/bin/bash
# A/B of one environment setting on one workload: alternating bench lines.
# Usage: env_ab.sh <outdir under gpurun_out> <workload> <steps> <reps> <VAR=value>
set -o pipefail
OUT=gpurun_out/$1; WL=$2; STEPS=$3; REPS=$4; KV=$5
mkdir -p $OUT
for rep in $(seq 1 $REPS); do
  for v in base var; do
    if [ $v = base ]; then E=FRECSYS_NONE=0; else E=$KV; fi
    env $E timeout -k 10 300 python bench.py --allow-env --workload $WL --extras= --cpu-seconds 0 --steps $STEPS --warmup 1 --quiet > $OUT/${WL}_${v}_$rep.json 2> $OUT/${WL}_${v}_$rep.err || { echo "$v failed"; tail -5 $OUT/${WL}_${v}_$rep.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['kernel_ms_per_epoch'];p=d['paths'];print(sys.argv[2], round(d['ms_per_step'],3), 'user', round(k['solve_user'],2), 'item', round(k['solve_item'],2), 'u-dspace TF', round(p['solve_user']['dspace_tflops'] or 0,1))" $OUT/${WL}_${v}_$rep.json ${WL}_${v}_$rep
  done
done
