#!/bin/bash
# One GPU round trip: the GPU test suite, the default bench line, and the
# N = 8 rank-0 / N = 1 kernel timelines of configs 2 and 4 (scripts/rank_share.py
# under rocprofv3 --kernel-trace; scripts/timeline_summary.py reads them).
# Usage: gpu_check.sh <outdir under gpurun_out> [tests|notests]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
mkdir -p $OUT
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; tail -30 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 2; }
echo bench ok
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/tr_ml20m_8_0 -o run --output-format csv -- python3 scripts/rank_share.py ials_ml20m_d256 3 8 0 > $OUT/tr_ml20m_8.log 2>&1 || { echo trace1 failed; exit 3; }
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/tr_ml20m_1_0 -o run --output-format csv -- python3 scripts/rank_share.py ials_ml20m_d256 3 1 0 > $OUT/tr_ml20m_1.log 2>&1 || { echo trace2 failed; exit 4; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr_msd_8_0 -o run --output-format csv -- python3 scripts/rank_share.py ials_msd_d512 3 8 0 > $OUT/tr_msd_8.log 2>&1 || { echo trace3 failed; exit 5; }
echo done
