#!/bin/bash
# A/B of library variants (ab/libfrecsys_hip_<v>.so, `make abvar`) on the MSD
# bench (config 4): alternating runs, ms per epoch and the d-space kernel times.
# Usage: msd_ab.sh <outdir under gpurun_out> <reps> <variant...>  (variant "base" = the tree's build)
# WL=<workload> (default ials_msd_d512), STEPS=<timed epochs> (default 3)
set -o pipefail
OUT=gpurun_out/$1; REPS=$2; shift 2
mkdir -p $OUT
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
cp $LIB $OUT/base.so.bak
trap 'cp $OUT/base.so.bak $LIB' EXIT
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    if [ $v = base ]; then cp $OUT/base.so.bak $LIB; else cp ab/libfrecsys_hip_$v.so $LIB; fi
    timeout -k 10 300 python bench.py --workload ${WL:-ials_msd_d512} --extras= --cpu-seconds 0 --steps ${STEPS:-3} --warmup 1 --quiet > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err || { echo "$v failed"; tail -5 $OUT/${v}_$rep.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['kernel_ms_per_epoch'];print(sys.argv[2], round(d['ms_per_step'],2), 'user dspace', round(k['solve_user.dspace'],2), 'item dspace', round(k['solve_item.dspace'],2))" $OUT/${v}_$rep.json ${v}_$rep
  done
done
