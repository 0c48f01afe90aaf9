set -o pipefail
OUT=gpurun_out/r4m
mkdir -p $OUT
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
cp $LIB $OUT/base.so.bak
cp ab/libfrecsys_hip_ablation.so $LIB
FRECSYS_DUAL_PROF=1 timeout -k 10 300 python bench.py --allow-env --workload ials_msd_d512 --extras= --cpu-seconds 0 --steps 2 --warmup 1 --quiet > $OUT/prof.json 2> $OUT/prof.err; rc=$?
cp $OUT/base.so.bak $LIB
rm -f $OUT/base.so.bak
grep "wide-prof" $OUT/prof.err | tail -16
exit $rc
