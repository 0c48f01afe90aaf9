#!/bin/bash
# Tests + serialized-stream kernel trace of bench.py (per-kernel times of one epoch).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
mkdir -p $OUT
if [ "$2" != "notest" ]; then
  timeout -k 10 500 python -m pytest tests/test_dual_gpu.py tests/test_parity_gpu.py tests/test_split_gpu.py -x -q > $OUT/tests.log 2>&1 || { echo tests failed; tail -30 $OUT/tests.log; exit 1; }
fi
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 > $OUT/bench.json 2> $OUT/bench.err || exit 2
FRECSYS_DUAL_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 > $OUT/trace.log 2>&1 || exit 3
echo ok
