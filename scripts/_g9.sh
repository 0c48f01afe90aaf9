# Wide SYRK overhead probe: MSD serialised kernel stats with the ablation
# library (FRECSYS_DEBUG_SKIP=1 drops the MFMAs; wrong numbers, timing only)
set -o pipefail
OUT=gpurun_out/r4g
mkdir -p $OUT
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
cp $LIB $OUT/base.so.bak
cp ab/libfrecsys_hip_ablation.so $LIB
for m in 0 1; do
  FRECSYS_DEBUG_SKIP=$m bash scripts/serial_prof.sh r4g/skip$m ials_msd_d512 2 > $OUT/skip$m.txt 2>&1 || { echo prof $m failed; tail -5 $OUT/skip$m.txt; cp $OUT/base.so.bak $LIB; exit 1; }
  echo "== skip $m"; grep -E "wide_syrk2|wide_chol|dual_solve_kernel<8|total" $OUT/skip$m.txt
done
cp $OUT/base.so.bak $LIB
rm -f $OUT/base.so.bak
