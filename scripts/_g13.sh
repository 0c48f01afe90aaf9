set -o pipefail
OUT=gpurun_out/r4k
mkdir -p $OUT
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
summ() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['kernel_ms_per_epoch'];print(sys.argv[2], round(d['ms_per_step'],2), {x: round(k[x],2) for x in ('solve_user','solve_item','solve_item.dspace','solve_item.split')})" $1 $2; }
for rep in 1 2; do
  for s in 4096 2048; do
    for w in ials_ml20m_d256 safer2_ml20m_d256; do
      FRECSYS_SPLIT_ROWS=$s timeout -k 10 300 python bench.py --allow-env --workload $w --extras= --cpu-seconds 0 --steps 10 --warmup 2 --quiet > $OUT/${w}_split${s}_$rep.json 2> $OUT/${w}_split${s}_$rep.err || { echo bench failed; exit 8; }
      summ $OUT/${w}_split${s}_$rep.json ${w}_split${s}_$rep
    done
  done
done
cp $LIB $OUT/new.so.bak
cp ab/libfrecsys_hip_ablation.so $LIB
for m in 0 1 1025; do
  FRECSYS_DEBUG_SKIP=$m bash scripts/serial_prof.sh r4k/skip$m ials_msd_d512 2 > $OUT/skip$m.txt 2>&1 || { echo prof $m failed; tail -5 $OUT/skip$m.txt; cp $OUT/new.so.bak $LIB; exit 1; }
  echo "== skip $m"; grep -E "wide_syrk2|total" $OUT/skip$m.txt
done
cp $OUT/new.so.bak $LIB
rm -f $OUT/new.so.bak
