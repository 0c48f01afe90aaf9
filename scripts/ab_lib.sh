#!/bin/bash
# A/B of library builds: GPU tests with the in-tree library, then bench.py
# ms_per_step + a serialised kernel trace per library.  Variant 1 is the
# in-tree libfrecsys_hip.so; each extra argument is another build of it
# (e.g. ab/libfrecsys_hip_old.so, made with an extra -D flag), swapped in
# for its run and swapped back at the end.
# Usage: ab_lib.sh <outdir> <tests|notest> [alt.so ...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
TESTS=$2
shift 2
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
mkdir -p $OUT
cp $LIB $OUT.main.so
if [ "$TESTS" != "notest" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo tests failed; tail -40 $OUT/tests.log; exit 1; }
fi
i=0
for v in "" "$@"; do
  i=$((i+1))
  if [ -n "$v" ]; then cp "$v" $LIB; else cp $OUT.main.so $LIB; fi
  timeout -k 10 240 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/bench_$i.json 2> $OUT/bench_$i.err || exit 2
  FRECSYS_DUAL_SERIAL=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_$i -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 > $OUT/trace_$i.log 2>&1 || exit 3
done
cp $OUT.main.so $LIB
rm -f $OUT.main.so
echo ok
