#!/bin/bash
# MSD-shaped iALS at d=512 (BASELINE configs[3] on one GPU): bench line +
# serialised per-kernel trace.  Usage: wide_prof.sh <outdir> [dim] [shape]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
DIM=${2:-512}
SHAPE=${3:-msd}
mkdir -p $OUT
timeout -k 10 400 python bench.py --shape $SHAPE --dim $DIM --reg 0.002 --uobs_weight 0.05 --steps 3 --warmup 1 --cpu-seconds 0 > $OUT/bench.json 2> $OUT/bench.err || exit 2
FRECSYS_DUAL_SERIAL=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --shape $SHAPE --dim $DIM --reg 0.002 --uobs_weight 0.05 --steps 1 --warmup 1 --cpu-seconds 0 > $OUT/trace.log 2>&1 || exit 3
echo ok
