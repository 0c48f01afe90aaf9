set -o pipefail
OUT=gpurun_out/r4j
mkdir -p $OUT
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
md5sum $LIB ab/libfrecsys_hip_oldring.so ab/libfrecsys_hip_ablation.so
cp $LIB $OUT/new.so.bak
restore() { cp $OUT/new.so.bak $LIB; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py tests/test_split_gpu.py tests/test_wide_split_gpu.py tests/test_models_gpu.py > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
summ() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['kernel_ms_per_epoch'];print(sys.argv[2], round(d['ms_per_step'],2), {x: round(k[x],2) for x in ('solve_user','solve_item','solve_user.dspace','solve_item.dspace')})" $1 $2; }
for rep in 1 2; do
  for v in new old; do
    if [ $v = old ]; then cp ab/libfrecsys_hip_oldring.so $LIB; else restore; fi
    for w in ials_msd_d512 safer2_ml20m_d256; do
      timeout -k 10 300 python bench.py --allow-env --workload $w --extras= --cpu-seconds 0 --steps 5 --warmup 2 --quiet > $OUT/${w}_${v}_$rep.json 2> $OUT/${w}_${v}_$rep.err || { echo bench failed; tail -5 $OUT/${w}_${v}_$rep.err; restore; exit 5; }
      summ $OUT/${w}_${v}_$rep.json ${w}_${v}_$rep
    done
  done
done
cp ab/libfrecsys_hip_ablation.so $LIB
for m in 1 1025 2049 3073; do
  FRECSYS_DEBUG_SKIP=$m bash scripts/serial_prof.sh r4j/skip$m ials_msd_d512 2 > $OUT/skip$m.txt 2>&1 || { echo prof $m failed; tail -5 $OUT/skip$m.txt; restore; exit 1; }
  echo "== skip $m"; grep -E "wide_syrk2|total" $OUT/skip$m.txt
done
restore
rm -f $OUT/new.so.bak
for rep in 1 2; do
  for s in 4096 2048; do
    FRECSYS_SPLIT_ROWS=$s timeout -k 10 300 python bench.py --allow-env --workload ials_ml20m_d256 --extras= --cpu-seconds 0 --steps 10 --warmup 2 --quiet > $OUT/ml20_split${s}_$rep.json 2> $OUT/ml20_split${s}_$rep.err || { echo bench failed; exit 8; }
    summ $OUT/ml20_split${s}_$rep.json ml20_split${s}_$rep
  done
done
