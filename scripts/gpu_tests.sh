#!/bin/bash
# Selected GPU test files, each in its own time-limited pytest process (so a
# hang names its file); stops at the first failure.
# Usage: gpu_tests.sh <outdir under gpurun_out> <test file...>
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for t in "$@"; do
  n=$(basename $t .py)
  timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread $t > $OUT/$n.log 2>&1; rc=$?
  echo "$n rc=$rc: $(tail -1 $OUT/$n.log)"
  [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $OUT/$n.log | head -20; exit $rc; }
done
exit 0
