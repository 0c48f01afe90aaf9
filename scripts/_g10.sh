set -o pipefail
OUT=gpurun_out/r4h
mkdir -p $OUT
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
md5sum $LIB ab/libfrecsys_hip_oldring.so
cp $LIB $OUT/new.so.bak
restore() { cp $OUT/new.so.bak $LIB; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_wide_split_gpu.py tests/test_wide_gpu.py tests/test_parity_gpu.py tests/test_sharded_gpu.py tests/test_split_gpu.py > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
summ() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));k=d['kernel_ms_per_epoch'];print(sys.argv[2], round(d['ms_per_step'],2), {x: round(k[x],2) for x in ('solve_user','solve_item','solve_user.dspace','solve_item.dspace')})" $1 $2; }
for rep in 1 2; do
  for v in new old wx6; do
    if [ $v = old ]; then cp ab/libfrecsys_hip_oldring.so $LIB; elif [ $v = wx6 ]; then cp ab/libfrecsys_hip_wx6.so $LIB; else restore; fi
    timeout -k 10 300 python bench.py --allow-env --workload ials_msd_d512 --extras= --cpu-seconds 0 --steps 5 --warmup 2 --quiet > $OUT/msd_${v}_$rep.json 2> $OUT/msd_${v}_$rep.err || { echo msd failed; tail -5 $OUT/msd_${v}_$rep.err; restore; exit 5; }
    summ $OUT/msd_${v}_$rep.json msd_${v}_$rep
  done
done
cp ab/libfrecsys_hip_wx6.so $LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_wide_split_gpu.py tests/test_wide_gpu.py tests/test_dual_gpu.py tests/test_config5_gpu.py > $OUT/pytest_wx6.log 2>&1; rc=$?
echo "wx6 pytest rc=$rc"; tail -2 $OUT/pytest_wx6.log
restore
[ $rc -ne 0 ] && exit $rc
bash scripts/_g9.sh
restore
for n in 2 4; do
  for s in 4096 2048; do
    FRECSYS_SPLIT_ROWS=$s timeout -k 10 240 python scripts/rank_share.py ials_ml20m_d256 5 $n > $OUT/rs_n${n}_split$s.jsonl 2> $OUT/rs_n${n}_split$s.err || { echo rs failed; tail -5 $OUT/rs_n${n}_split$s.err; exit 7; }
    echo "N=$n split_rows=$s $(tail -1 $OUT/rs_n${n}_split$s.jsonl)"
  done
done
rm -f $OUT/new.so.bak
for cfg in "224 2048" "0 2048" "0 4096" "128 2048"; do
  set -- $cfg
  FRECSYS_DUAL_MAX_H_ITEM=$1 FRECSYS_SPLIT_ROWS=$2 timeout -k 10 240 python scripts/rank_share.py ials_ml20m_d256 5 8 > $OUT/rs_item$1_split$2.jsonl 2> $OUT/rs_item$1_split$2.err || { echo rs failed; tail -5 $OUT/rs_item$1_split$2.err; exit 7; }
  echo "item_max_h=$1 split_rows=$2 $(tail -1 $OUT/rs_item$1_split$2.jsonl)"
done
