#!/bin/bash
# A/B of library builds on one bench workload (no tests): sec/epoch and the
# serialised times of the kernels matching a pattern, per library (each
# alternative swapped in for its run, the in-tree one restored).
# Usage: ab_kern.sh <outdir> <workload> <kernel regex> [alt.so ...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
W=$2
PAT=$3
shift 3
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
mkdir -p $OUT
cp $LIB /tmp/libfrecsys_hip.main.so
trap 'cp /tmp/libfrecsys_hip.main.so $LIB' EXIT
i=0
for v in "" "$@"; do
  i=$((i+1))
  if [ -n "$v" ]; then cp "$v" $LIB; else cp /tmp/libfrecsys_hip.main.so $LIB; fi
  timeout -k 10 240 python bench.py --workload $W --extras= --steps 5 --warmup 2 --cpu-seconds 0 --quiet > $OUT/bench_$i.json 2> $OUT/bench_$i.err || exit 2
  FRECSYS_DUAL_SERIAL=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_$i -o run --output-format csv -- python3 bench.py --workload $W --extras= --allow-env --steps 1 --warmup 0 --cpu-seconds 0 --quiet > $OUT/trace_$i.log 2>&1 || exit 3
  echo "== variant $i ${v:-in-tree}: sec/epoch $(python3 -c "import json; print(round(json.load(open('$OUT/bench_$i.json'))['sec_per_epoch'], 5))")"
  python3 scripts/kstats.py $OUT/trace_$i/run_kernel_stats.csv 1 | grep -E "$PAT|total"
done
