#!/bin/bash
# Round-5 closing pass on one GPU box: the whole -m gpu suite, smoke(), the
# default bench line, config 5's kernel stats + FETCH / WRITE passes, and one
# ablation-build run with a mask that used to abort (NOT_SPD on garbage A).
# Usage: final_r05.sh <outdir under gpurun_out>
set -o pipefail
OUT=gpurun_out/${1:-final_r05}
mkdir -p $OUT
bash scripts/final_check.sh ${1:-final_r05} || exit 1
bash scripts/config5_prof.sh ${1:-final_r05}/c5 skip-bench || exit 2
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
cp $LIB $OUT/base.so.bak
trap 'cp $OUT/base.so.bak $LIB; rm -f $OUT/base.so.bak' EXIT
cp ab/libfrecsys_hip_ablation.so $LIB
FRECSYS_DEBUG_SKIP=2049 timeout -k 10 300 python bench.py --allow-env --workload ials_msd_d512 --extras= --cpu-seconds 0 --steps 1 --warmup 1 --quiet > $OUT/ablation_2049.json 2> $OUT/ablation_2049.err; rc=$?
echo "ablation FRECSYS_DEBUG_SKIP=2049 rc=$rc"
[ $rc -eq 0 ] || tail -5 $OUT/ablation_2049.err
exit $rc
