#!/bin/bash
# One SQ counter pass (MFMA busy, active / issue-stalled / parked wave cycles,
# instruction mix) over one bench workload, streams serialised; summarised per
# kernel by scripts/sq_summary.py.
# Usage: sq_workload.sh <outdir under gpurun_out> <workload>
set -o pipefail
OUT=gpurun_out/$1; WL=$2
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
FRECSYS_DUAL_SERIAL=1 timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/pmc -o run --output-format csv -- python3 bench.py --workload $WL --extras= --cpu-seconds 0 --allow-env --steps 1 --warmup 1 --quiet > $OUT/pmc.log 2>&1 || { echo pmc failed; tail -5 $OUT/pmc.log; exit 1; }
python3 scripts/sq_summary.py $OUT/pmc/run_counter_collection.csv 256 $OUT/sq.json > $OUT/sq.txt
head -24 $OUT/sq.txt
