#!/bin/bash
# Kernel stats of config 5 for library variants (ab/libfrecsys_hip_<v>.so,
# "tree" = the tree's library): the wide Cholesky kernels' average launch.
# Usage: chol2_var.sh <outdir under gpurun_out> <variant...>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift
W=safer2_2m500k_d1024
mkdir -p $OUT
ARGS="--allow-env --workload $W --extras= --steps 2 --warmup 1 --cpu-seconds 0"
for v in "$@"; do
  if [ $v = tree ]; then RUN=""; else RUN="bash scripts/with_lib.sh $v"; fi
  FRECSYS_DUAL_SERIAL=${SERIAL:-0} timeout -s KILL 300 $RUN rocprofv3 --kernel-trace --stats -d $OUT/trace_$v -o run --output-format csv -- python3 -u bench.py $ARGS > $OUT/trace_$v.log 2>&1 || { echo trace $v failed; exit 2; }
  python3 scripts/kstats.py $OUT/trace_$v/run_kernel_stats.csv 2 > $OUT/kstats_$v.txt || { echo kstats failed; exit 3; }
  echo "== $v $(grep -E 'wide_chol2|wide_chol_kernel<32' $OUT/kstats_$v.txt | head -1 | cut -c1-20,60-)"
done
