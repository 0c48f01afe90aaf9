#!/bin/bash
# SQ stall breakdown of bench.py's kernels (one --pmc pass, no tracing domains).
# Usage: pmc_sq2.sh <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
mkdir -p $OUT
FRECSYS_DUAL_SERIAL=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/pmc -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 > $OUT/pmc.log 2>&1 || exit 3
echo ok
