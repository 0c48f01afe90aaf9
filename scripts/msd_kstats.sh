#!/bin/bash
# MSD (config 4, d = 512) rocprofv3 kernel stats, streams serialised (no PMC).
# Usage: msd_kstats.sh <outdir under gpurun_out> [extra env assignments...]
set -o pipefail
OUT=gpurun_out/$1
shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
for kv in "$@"; do export "$kv"; done
FRECSYS_DUAL_SERIAL=1 timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --workload ials_msd_d512 --extras= --cpu-seconds 0 --allow-env --steps 2 --warmup 1 --quiet > $OUT/trace.log 2>&1 || { echo trace failed; tail -5 $OUT/trace.log; exit 1; }
python3 scripts/kstats.py $OUT/trace/run_kernel_stats.csv 3 | tee $OUT/kstats.txt
