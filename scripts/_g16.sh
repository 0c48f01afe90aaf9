set -o pipefail
OUT=gpurun_out/r4n
mkdir -p $OUT
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
cp $LIB $OUT/base.so.bak
restore() { cp $OUT/base.so.bak $LIB; }
for v in cmb1 cmb2; do
  cp ab/libfrecsys_hip_$v.so $LIB
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_wide_split_gpu.py tests/test_wide_gpu.py tests/test_sharded_gpu.py tests/test_config5_gpu.py > $OUT/pytest_$v.log 2>&1; rc=$?
  echo "$v pytest rc=$rc"; tail -2 $OUT/pytest_$v.log
  [ $rc -ne 0 ] && { restore; exit $rc; }
done
summ() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['kernel_ms_per_epoch'];print(sys.argv[2], round(d['ms_per_step'],2), {x: round(k[x],2) for x in ('solve_user','solve_item','solve_user.dspace','solve_item.dspace')})" $1 $2; }
for rep in 1 2; do
  for v in base cmb1 cmb2; do
    if [ $v = base ]; then restore; else cp ab/libfrecsys_hip_$v.so $LIB; fi
    timeout -k 10 300 python bench.py --allow-env --workload ials_msd_d512 --extras= --cpu-seconds 0 --steps 5 --warmup 2 --quiet > $OUT/msd_${v}_$rep.json 2> $OUT/msd_${v}_$rep.err || { echo bench failed; tail -5 $OUT/msd_${v}_$rep.err; restore; exit 5; }
    summ $OUT/msd_${v}_$rep.json msd_${v}_$rep
  done
done
for v in cmb1 cmb2; do
  cp ab/libfrecsys_hip_$v.so $LIB
  bash scripts/serial_prof.sh r4n/ser_$v ials_msd_d512 2 > $OUT/ser_$v.txt 2>&1 || { echo prof failed; restore; exit 6; }
  echo "== $v"; grep -E "wide_syrk2|total" $OUT/ser_$v.txt
done
restore
rm -f $OUT/base.so.bak
