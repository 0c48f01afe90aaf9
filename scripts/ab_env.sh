#!/bin/bash
# A/B of an environment switch: GPU tests (with the default env), then
# bench.py ms_per_step and a serialised kernel trace per variant.
# Usage: ab_env.sh <outdir> <tests|notest> "<ENV=VAL ...>" ["<ENV=VAL ...>" ...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
TESTS=$2
shift 2
mkdir -p $OUT
if [ "$TESTS" != "notest" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread $TESTS_ARGS > $OUT/tests.log 2>&1 || { echo tests failed; tail -40 $OUT/tests.log; exit 1; }
fi
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 240 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/bench_$i.json 2> $OUT/bench_$i.err || exit 2
  env $v FRECSYS_DUAL_SERIAL=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_$i -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 > $OUT/trace_$i.log 2>&1 || exit 3
done
echo ok
