#!/bin/bash
# Phase cycles and ablations of the wide SYRK (ablation build, MSD, streams
# serialised).  Usage: w3_ablate.sh <outdir under gpurun_out> <mask...>
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
cp $LIB $OUT/base.so.bak
trap 'cp $OUT/base.so.bak $LIB' EXIT
cp ab/libfrecsys_hip_ablation.so $LIB
for m in "$@"; do
  FRECSYS_DEBUG_SKIP=$m FRECSYS_DUAL_SERIAL=1 FRECSYS_DUAL_PROF=1 timeout -k 10 200 python bench.py --allow-env --workload ials_msd_d512 --extras= --cpu-seconds 0 --steps 1 --warmup 1 --quiet > $OUT/m$m.json 2> $OUT/m$m.err || { echo "mask $m failed"; tail -5 $OUT/m$m.err; exit 1; }
  echo "== mask $m: $(python3 -c "import json;d=json.load(open('$OUT/m$m.json'));k=d['kernel_ms_per_epoch'];print('epoch',round(d['ms_per_step'],2),'item dspace',round(k['solve_item.dspace'],2),'user dspace',round(k['solve_user.dspace'],2))")"
  grep "wide-prof" $OUT/m$m.err | tail -8
done
