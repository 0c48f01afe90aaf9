#!/bin/bash
# Measurement pass for the round: bench line + rocprofv3 kernel stats + PMC
# traffic passes (separate runs, never combined with tracing domains).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $OUT/trace.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 > $OUT/pmc_fetch.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --cpu-seconds 0 > $OUT/pmc_write.log 2>&1 || exit 4
echo done
