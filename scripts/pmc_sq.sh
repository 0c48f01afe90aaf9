#!/bin/bash
# SQ counters of bench.py's kernels (one --pmc pass, no tracing domains).
# Usage: pmc_sq.sh <outdir> [extra env]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
mkdir -p $OUT
env ${2:-FRECSYS_X=0} FRECSYS_DUAL_SERIAL=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU -d $OUT/pmc -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 > $OUT/pmc.log 2>&1 || exit 3
echo ok
