#!/bin/bash
# SQ counters of the wide Cholesky kernels at config 5 (two-panel default and
# FRECSYS_WIDE_CHOL2=0), one rocprofv3 --pmc pass per counter set.
# Usage: chol2_sq.sh <outdir under gpurun_out>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
W=safer2_2m500k_d1024
mkdir -p $OUT
ARGS="--allow-env --workload $W --extras= --steps 1 --warmup 0 --cpu-seconds 0"
S1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS"
S2="SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES"
for v in 1 0; do
  for k in 1 2; do
    eval CS=\$S$k
    FRECSYS_WIDE_CHOL2=$v timeout -s KILL 300 rocprofv3 --pmc $CS --kernel-include-regex wide_chol -d $OUT/sq${k}_$v -o run --output-format csv -- python3 -u bench.py $ARGS > $OUT/sq${k}_$v.log 2>&1 || { echo sq$k $v failed; tail -5 $OUT/sq${k}_$v.log; exit 2; }
  done
  python3 scripts/sq_summary.py $OUT/sq1_$v/run_counter_collection.csv 256 > $OUT/sq1_$v.txt
  echo "== chol2=$v"; cat $OUT/sq1_$v.txt
  python3 - $OUT/sq2_$v/run_counter_collection.csv <<'PY'
import csv,sys,collections
acc=collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    n=r["Kernel_Name"].split("(anonymous namespace)::")[-1].split("(")[0]
    acc[n][r["Counter_Name"]]+=float(r["Counter_Value"])
for n,c in acc.items():
    print(n, {k: f"{v:.4g}" for k,v in c.items()})
PY
done
