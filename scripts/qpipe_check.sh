#!/bin/bash
# GPU check of the pipelined form-Q (Q rows formed inside the tridiagonal
# reduction's launch): the basis / history-space / eager / sharded tests,
# the per-rank epochs at N = 8 of configs 2 and 4, the default bench line,
# and the headline kernel trace (10 steps) for the roofline cross-check.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dual_gpu.py tests/test_wide_gpu.py tests/test_eager_gpu.py tests/test_sharded_gpu.py tests/test_comm_gpu.py > $OUT/pytest.log 2>&1 || { echo pytest failed; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python scripts/rank_share.py ials_ml20m_d256 5 8 > $OUT/c2_n8.jsonl || { echo rs2 failed; exit 2; }
tail -1 $OUT/c2_n8.jsonl
timeout -k 10 300 python scripts/rank_share.py ials_msd_d512 3 8 > $OUT/c4_n8.jsonl || { echo rs4 failed; exit 3; }
tail -1 $OUT/c4_n8.jsonl
timeout -k 10 420 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; exit 4; }
echo bench ok
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_ials_ml20m_d256 -o run --output-format csv -- python3 bench.py --workload ials_ml20m_d256 --extras= --steps 10 --warmup 1 --cpu-seconds 0 --quiet > $OUT/trace.log 2>&1 || { echo trace failed; exit 5; }
echo done
