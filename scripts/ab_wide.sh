#!/bin/bash
# A/B of library builds on one bench workload: wide tests with the in-tree
# library, then sec/epoch and the serialised wide kernel times per library
# (each alternative swapped in for its run, the in-tree one restored).
# Usage: ab_wide.sh <outdir> <workload> [alt.so ...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
W=$2
shift 2
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
mkdir -p $OUT
cp $LIB /tmp/libfrecsys_hip.main.so
trap 'cp /tmp/libfrecsys_hip.main.so $LIB' EXIT
i=0
for v in "" "$@"; do
  i=$((i+1))
  if [ -n "$v" ]; then cp "$v" $LIB; else cp /tmp/libfrecsys_hip.main.so $LIB; fi
  timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_wide_gpu.py tests/test_workload_gpu.py -k "wide or msd or slice" > $OUT/tests_$i.log 2>&1 || { echo "variant $i ($v) tests failed"; tail -20 $OUT/tests_$i.log; exit 1; }
  timeout -k 10 240 python bench.py --workload $W --extras= --steps 3 --warmup 1 --cpu-seconds 0 --quiet > $OUT/bench_$i.json 2> $OUT/bench_$i.err || exit 2
  FRECSYS_DUAL_SERIAL=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_$i -o run --output-format csv -- python3 bench.py --workload $W --extras= --allow-env --steps 1 --warmup 0 --cpu-seconds 0 --quiet > $OUT/trace_$i.log 2>&1 || exit 3
  echo "== variant $i ${v:-in-tree}: $(tail -1 $OUT/tests_$i.log)"
  python3 -c "import json; l=json.load(open('$OUT/bench_$i.json')); print('sec/epoch', round(l['sec_per_epoch'],4))"
  python3 scripts/kstats.py $OUT/trace_$i/run_kernel_stats.csv 1 | grep -E "wide_chol|wide_syrk2_kernel<1>|total"
done
