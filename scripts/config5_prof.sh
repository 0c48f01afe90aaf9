#!/bin/bash
# Config 5 (2M x 500K, d = 1024, SAFER2) measurement pass on the GPU box:
#   1. the default bench line (headline + extras, config 5 included at N=1)
#   2. rocprofv3 kernel stats of config 5 alone (2 timed epochs)
#   3. FETCH_SIZE and WRITE_SIZE passes (separate runs, no tracing domains),
#      summarised by scripts/pmc_summary.py into <out>/latest_pmc.json
# Usage: config5_prof.sh <outdir under gpurun_out> [skip-bench]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
W=safer2_2m500k_d1024
mkdir -p $OUT
if [ -z "$2" ]; then
  timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; exit 1; }
  echo "bench ok"
fi
ARGS="--workload $W --extras= --steps 2 --warmup 1 --cpu-seconds 0"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$W -o run --output-format csv -- python3 -u bench.py $ARGS > $OUT/trace_$W.log 2>&1 || { echo trace failed; exit 2; }
python3 scripts/kstats.py $OUT/trace_$W/run_kernel_stats.csv 2 > $OUT/kstats_$W.txt || { echo kstats failed; exit 3; }
PARGS="--workload $W --extras= --steps 1 --warmup 1 --cpu-seconds 0"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_$W -o run --output-format csv -- python3 -u bench.py $PARGS > $OUT/fetch_$W.log 2>&1 || { echo fetch failed; exit 4; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write_$W -o run --output-format csv -- python3 -u bench.py $PARGS > $OUT/write_$W.log 2>&1 || { echo write failed; exit 5; }
python3 scripts/pmc_summary.py $W $OUT/fetch_$W/run_counter_collection.csv $OUT/write_$W/run_counter_collection.csv 2 $OUT/pmc_$W.json $OUT/latest_pmc.json > $OUT/pmc_$W.txt || { echo summary failed; exit 6; }
echo done
