#!/bin/bash
# Alternating bench lines of one workload with an environment switch at
# each of its values.  Usage: env_ab.sh <outdir> <workload> <steps> <reps> <VAR> <values...>
set -o pipefail
OUT=gpurun_out/$1 W=$2 ST=$3 REPS=$4 VAR=$5
shift 5
mkdir -p $OUT
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 400 python bench.py --allow-env --workload $W --extras= --cpu-seconds 0 --steps $ST --warmup 1 --quiet > $OUT/${W}_${v}_$rep.json 2> $OUT/${W}_${v}_$rep.err || { echo "bench $W $v failed"; tail -5 $OUT/${W}_${v}_$rep.err; exit 5; }
    python3 -c "
import json,sys
d=json.load(open(sys.argv[1]));k=d.get('kernel_ms_per_epoch',{})
print(sys.argv[2], round(d['ms_per_step'],2), ' '.join(f'{n}={k[n]:.1f}' for n in ('solve_user','solve_item','solve_item.dspace') if n in k))" $OUT/${W}_${v}_$rep.json ${VAR}=${v}_$rep
  done
done
