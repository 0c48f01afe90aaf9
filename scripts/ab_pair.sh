#!/bin/bash
# A/B of one alternative wide library: bit-for-bit outputs vs the in-tree
# build, the wide tests with it, then MSD sec/epoch + serialised wide kernels
# for both.  Usage: ab_pair.sh <outdir> <alt.so>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
ALT=$2
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
mkdir -p $OUT
cp $LIB /tmp/libfrecsys_hip.main.so
trap 'cp /tmp/libfrecsys_hip.main.so $LIB' EXIT
timeout -k 10 120 python scripts/dbg/wide_dump.py $OUT/main.npz > $OUT/dump_main.log 2>&1 || { echo dump main failed; tail $OUT/dump_main.log; exit 1; }
cp $ALT $LIB
timeout -k 10 120 python scripts/dbg/wide_dump.py $OUT/alt.npz > $OUT/dump_alt.log 2>&1 || { echo dump alt failed; tail $OUT/dump_alt.log; exit 1; }
python3 -c "
import numpy as np
a=np.load('$OUT/main.npz'); b=np.load('$OUT/alt.npz')
for k in a.files: print(k, 'bit-identical' if np.array_equal(a[k], b[k]) else 'DIFFERS max %g' % np.abs(a[k]-b[k]).max())
"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_wide_split_gpu.py tests/test_wide_gpu.py > $OUT/tests_alt.log 2>&1 || { echo "alt tests failed"; tail -30 $OUT/tests_alt.log; exit 1; }
tail -1 $OUT/tests_alt.log
i=0
for v in /tmp/libfrecsys_hip.main.so $ALT; do
  i=$((i+1))
  cp $v $LIB
  timeout -k 10 240 python bench.py --workload ials_msd_d512 --extras= --steps 3 --warmup 1 --cpu-seconds 0 --quiet > $OUT/bench_$i.json 2> $OUT/bench_$i.err || exit 2
  FRECSYS_DUAL_SERIAL=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_$i -o run --output-format csv -- python3 bench.py --workload ials_msd_d512 --extras= --allow-env --steps 1 --warmup 0 --cpu-seconds 0 --quiet > $OUT/trace_$i.log 2>&1 || exit 3
  echo "== variant $i $v: sec/epoch $(python3 -c "import json; print(round(json.load(open('$OUT/bench_$i.json'))['sec_per_epoch'], 5))")"
  python3 scripts/kstats.py $OUT/trace_$i/run_kernel_stats.csv 1 | grep -E "wide_chol|wide_syrk2|total"
done
