#!/bin/bash
# Serialised-stream rocprofv3 kernel stats of one bench.py workload.
# Usage: serial_prof.sh <outdir under gpurun_out> <workload> [steps]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
W=$2
S=${3:-2}
mkdir -p $OUT
FRECSYS_DUAL_SERIAL=1 timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --workload $W --extras= --cpu-seconds 0 --allow-env --steps $S --warmup 1 --quiet > $OUT/trace.log 2>&1 || { echo trace failed; tail -5 $OUT/trace.log; exit 1; }
python3 scripts/kstats.py $OUT/trace/run_kernel_stats.csv $((S + 1))
