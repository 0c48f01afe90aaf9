#!/bin/bash
# Config 5 kernel stats with the streams serialised (3 epochs: warmup + 2).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5k5
mkdir -p $OUT
FRECSYS_DUAL_SERIAL=1 timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --allow-env --workload safer2_2m500k_d1024 --extras= --cpu-seconds 0 --steps 2 --warmup 1 --quiet > $OUT/trace.log 2>&1 || { echo trace failed; exit 1; }
python3 scripts/kstats.py $OUT/trace/run_kernel_stats.csv 3 30 > $OUT/kstats.txt
cat $OUT/kstats.txt
