#!/bin/bash
# What bounds the user half-step's d-space stream at the wide dims: for each
# workload, the bench line with the streams overlapped (default) and
# serialised (FRECSYS_DUAL_SERIAL=1), then a serialised kernel trace whose
# last epoch scripts/timeline_summary.py lists launch by launch.
# Usage: user_dspace_prof.sh <outdir under gpurun_out> <workload...>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
shift
mkdir -p $OUT
for w in "$@"; do
  timeout -k 10 300 python bench.py --workload $w --extras= --cpu-seconds 0 --steps 3 --warmup 1 --quiet > $OUT/${w}_overlap.json 2> $OUT/${w}_overlap.err || { echo bench $w failed; exit 1; }
  FRECSYS_DUAL_SERIAL=1 timeout -k 10 300 python bench.py --allow-env --workload $w --extras= --cpu-seconds 0 --steps 3 --warmup 1 --quiet > $OUT/${w}_serial.json 2> $OUT/${w}_serial.err || { echo serial bench $w failed; exit 2; }
  FRECSYS_DUAL_SERIAL=1 timeout -s KILL 300 rocprofv3 --kernel-trace -d $OUT/trace_$w -o run --output-format csv -- python3 bench.py --allow-env --workload $w --extras= --cpu-seconds 0 --steps 1 --warmup 1 --quiet > $OUT/trace_$w.log 2>&1 || { echo trace $w failed; exit 3; }
  python3 scripts/timeline_summary.py $OUT/trace_$w/run_kernel_trace.csv loss_gather $OUT/timeline_$w.json > $OUT/timeline_$w.txt || { echo timeline $w failed; exit 4; }
  echo "$w ok"
done
