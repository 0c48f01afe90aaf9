#!/bin/bash
# Round-6 A/B of library variants on one GPU box: a bitwise check of each
# variant against the first one (two iALS epochs at d = 64..512, ML-20M-like
# quirk data: scripts/bitwise_epochs.py), optional GPU tests on each variant,
# then alternating bench lines over the workloads.
# Usage: ab_r06.sh <outdir under gpurun_out> <reps> <variant...>
#   variant "tree" = the library in the tree, otherwise ab/libfrecsys_hip_<v>.so
#   TESTS run on "tree" only.
#   WLS="ials_ml20m_d256 ials_msd_d512 safer2_2m500k_d1024" (default), TESTS="tests/..." (default none)
#   BITWISE=0 skips the bitwise check (variants that change rounding)
set -o pipefail
OUT=gpurun_out/$1; REPS=$2; shift 2
mkdir -p $OUT
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
cp $LIB $OUT/tree.so.bak
restore() { cp $OUT/tree.so.bak $LIB; }
trap 'restore; rm -f $OUT/tree.so.bak' EXIT
use() { if [ $1 = tree ]; then restore; else cp ab/libfrecsys_hip_$1.so $LIB; fi; }
first=$1
if [ "${BITWISE:-1}" = 1 ]; then
  for v in "$@"; do
    use $v
    timeout -k 10 300 python -u scripts/bitwise_epochs.py $OUT/bw_$v.npz > $OUT/bw_$v.log 2>&1 || { echo "bitwise $v failed"; tail -5 $OUT/bw_$v.log; exit 3; }
    python3 -c "
import numpy as np,sys
a=np.load(sys.argv[1]);b=np.load(sys.argv[2])
bad=[k for k in a.files if not np.array_equal(a[k],b[k])]
print('bitwise', sys.argv[3], 'vs', sys.argv[4], 'identical' if not bad else 'DIFFER '+str(bad))" $OUT/bw_$first.npz $OUT/bw_$v.npz $v $first
  done
fi
if [ -n "$TESTS" ]; then
  for v in "$@"; do
    [ $v = tree ] || continue
    use $v
    timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > $OUT/pytest_$v.log 2>&1; rc=$?
    echo "$v pytest rc=$rc: $(tail -1 $OUT/pytest_$v.log)"
    [ $rc -ne 0 ] && { tail -30 $OUT/pytest_$v.log; exit 4; }
  done
fi
for rep in $(seq 1 $REPS); do
  for w in ${WLS:-ials_ml20m_d256 ials_msd_d512 safer2_2m500k_d1024}; do
    st=20; [ $w = ials_msd_d512 ] && st=5; [ $w = safer2_2m500k_d1024 ] && st=2
    for v in "$@"; do
      use $v
      timeout -k 10 400 python bench.py --allow-env --workload $w --extras= --cpu-seconds 0 --steps $st --warmup 1 --quiet > $OUT/${w}_${v}_$rep.json 2> $OUT/${w}_${v}_$rep.err || { echo "bench $w $v failed"; tail -5 $OUT/${w}_${v}_$rep.err; exit 5; }
      python3 -c "
import json,sys
d=json.load(open(sys.argv[1]));k=d.get('kernel_ms_per_epoch',{})
print(sys.argv[2], round(d['ms_per_step'],2), ' '.join(f'{n}={k[n]:.1f}' for n in ('solve_user','solve_item','solve_user.hspace','solve_item.hspace','solve_user.dspace','solve_item.dspace') if n in k))" $OUT/${w}_${v}_$rep.json ${w}_${v}_$rep
    done
  done
done
