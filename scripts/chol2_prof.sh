#!/bin/bash
# Kernel stats of config 5 with the two-panel wide Cholesky (default) and
# the one-panel kernel (FRECSYS_WIDE_CHOL2=0); VALS: the values, SERIAL=1:
# streams serialised.
# Usage: chol2_prof.sh <outdir under gpurun_out>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
W=safer2_2m500k_d1024
mkdir -p $OUT
ARGS="--allow-env --workload $W --extras= --steps 2 --warmup 1 --cpu-seconds 0"
for v in ${VALS:-1 0}; do
  FRECSYS_DUAL_SERIAL=${SERIAL:-0} FRECSYS_WIDE_CHOL2=$v timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$v -o run --output-format csv -- python3 -u bench.py $ARGS > $OUT/trace_$v.log 2>&1 || { echo trace $v failed; exit 2; }
  python3 scripts/kstats.py $OUT/trace_$v/run_kernel_stats.csv 2 > $OUT/kstats_$v.txt || { echo kstats failed; exit 3; }
  echo "== chol2=$v"; grep -E "wide_chol|total" $OUT/kstats_$v.txt
done
