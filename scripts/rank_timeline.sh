#!/bin/bash
# Kernel timeline of one rank's share (scripts/rank_share.py <wl> <steps> <N> <rank>)
# under rocprofv3 --kernel-trace, summarised by scripts/timeline_summary.py.
# Usage: rank_timeline.sh <outdir under gpurun_out> <workload> <N> <rank>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; WL=$2; N=$3; R=$4
mkdir -p $OUT
timeout -s KILL 300 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- python3 scripts/rank_share.py $WL 3 $N $R > $OUT/rs.jsonl 2> $OUT/rs.err || { echo trace failed; exit 1; }
python3 scripts/timeline_summary.py $OUT/trace/run_kernel_trace.csv loss_gather $OUT/timeline.json > $OUT/timeline.txt || exit 2
tail -1 $OUT/timeline.txt
