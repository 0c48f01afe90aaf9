#!/bin/bash
# A/B of one alternative library against the in-tree build: bit-for-bit
# outputs (scripts/dbg/wide_dump.py, d = 128..1000), the whole GPU test suite
# with the in-tree build, then per library the bench sec/epoch of the given
# workloads and the serialised kernel stats of the first.
# Usage: ab_head.sh <outdir> <alt.so> <workload> [workload ...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
ALT=$2
shift 2
W0=$1
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
mkdir -p $OUT
cp $LIB /tmp/libfrecsys_hip.main.so
trap 'cp /tmp/libfrecsys_hip.main.so $LIB' EXIT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 120 python scripts/dbg/wide_dump.py $OUT/main.npz > $OUT/dump_main.log 2>&1 || { echo dump main failed; tail $OUT/dump_main.log; exit 1; }
cp $ALT $LIB
timeout -k 10 120 python scripts/dbg/wide_dump.py $OUT/alt.npz > $OUT/dump_alt.log 2>&1 || { echo dump alt failed; tail $OUT/dump_alt.log; exit 1; }
python3 -c "
import numpy as np
a=np.load('$OUT/main.npz'); b=np.load('$OUT/alt.npz')
for k in a.files: print(k, 'bit-identical' if np.array_equal(a[k], b[k]) else 'DIFFERS max %g' % np.abs(a[k]-b[k]).max())
"
i=0
for v in /tmp/libfrecsys_hip.main.so $ALT; do
  i=$((i+1))
  cp $v $LIB
  for W in "$@"; do
    timeout -k 10 240 python bench.py --workload $W --extras= --steps 5 --warmup 2 --cpu-seconds 0 --quiet > $OUT/bench_${i}_$W.json 2> $OUT/bench_${i}_$W.err || exit 2
    echo "== variant $i $v $W: sec/epoch $(python3 -c "import json; print(round(json.load(open('$OUT/bench_${i}_$W.json'))['sec_per_epoch'], 5))")"
  done
  FRECSYS_DUAL_SERIAL=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_$i -o run --output-format csv -- python3 bench.py --workload $W0 --extras= --allow-env --steps 1 --warmup 0 --cpu-seconds 0 --quiet > $OUT/trace_$i.log 2>&1 || exit 3
  python3 scripts/kstats.py $OUT/trace_$i/run_kernel_stats.csv 1 8
done
