#!/bin/bash
# One rocprofv3 --pmc pass over the MSD bench (config 4, streams serialised).
# Usage: msd_pmc.sh <outdir under gpurun_out> "<counters>" [extra env assignments...]
set -o pipefail
OUT=gpurun_out/$1
CTRS=$2
shift 2
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
for kv in "$@"; do export "$kv"; done
FRECSYS_DUAL_SERIAL=1 timeout -s KILL 120 rocprofv3 --pmc $CTRS -d $OUT/pmc -o run --output-format csv -- python3 bench.py --workload ials_msd_d512 --extras= --cpu-seconds 0 --allow-env --steps 1 --warmup 1 --quiet > $OUT/pmc.log 2>&1 || { echo pmc failed; tail -5 $OUT/pmc.log; exit 1; }
python3 scripts/pmc_raw.py $OUT/pmc/run_counter_collection.csv wide_syrk wide_chol | tee $OUT/pmc.txt
