#!/bin/bash
# Counter-measured gather traffic of one half-step (the north-star figure on
# a table larger than the Infinity Cache: the MSD item half-step gathers the
# 0.97 GB user table), plus the FETCH_SIZE calibration of the access widths.
# Usage: gather_prof.sh <outdir under gpurun_out> [workload] [side]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
W=${2:-ials_msd_d512}
S=${3:-item}
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_cal -o run --output-format csv -- ./scripts/micro/fetch_cal > $OUT/fetch_cal.log 2>&1 || { echo fetch_cal failed; exit 1; }
timeout -k 10 300 python3 scripts/halfstep_probe.py $W $S 2 > $OUT/probe.json 2> $OUT/probe.err || { echo probe failed; exit 2; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 scripts/halfstep_probe.py $W $S 2 > $OUT/fetch.log 2>&1 || { echo fetch pass failed; exit 3; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 scripts/halfstep_probe.py $W $S 2 > $OUT/write.log 2>&1 || { echo write pass failed; exit 4; }
echo done
