#!/bin/bash
# Serialised kernel trace of bench.py under FRECSYS_DEBUG_SKIP ablation masks
# (results are garbage under a mask; only the kernel times are read).
# Usage: ablate_trace.sh <outdir> <mask> [<mask> ...]
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
shift
mkdir -p $OUT
for m in "$@"; do
  FRECSYS_DEBUG_SKIP=$m FRECSYS_DUAL_SERIAL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace_$m -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 > $OUT/trace_$m.log 2>&1
done
echo done
