#!/bin/bash
# Wide-path A/B: the wide GPU tests (incl. the slab split) with the in-tree
# library, then per library the MSD bench sec/epoch and the serialised wide
# kernel times.  Usage: ab_wide2.sh <outdir> <workload> [alt.so ...]
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
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_wide_split_gpu.py tests/test_wide_gpu.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
i=0
for v in "" "$@"; do
  i=$((i+1))
  if [ -n "$v" ]; then cp "$v" $LIB; else cp /tmp/libfrecsys_hip.main.so $LIB; fi
  timeout -k 10 240 python bench.py --workload $W --extras= --steps 3 --warmup 1 --cpu-seconds 0 --quiet > $OUT/bench_$i.json 2> $OUT/bench_$i.err || exit 2
  FRECSYS_DUAL_SERIAL=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_$i -o run --output-format csv -- python3 bench.py --workload $W --extras= --allow-env --steps 1 --warmup 0 --cpu-seconds 0 --quiet > $OUT/trace_$i.log 2>&1 || exit 3
  echo "== variant $i ${v:-in-tree}: sec/epoch $(python3 -c "import json; print(round(json.load(open('$OUT/bench_$i.json'))['sec_per_epoch'], 5))")"
  python3 scripts/kstats.py $OUT/trace_$i/run_kernel_stats.csv 1 | grep -E "wide_chol|wide_syrk2|total"
done
