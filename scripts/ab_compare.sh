# usage: bash scripts/ab_compare.sh <outdir under gpurun_out> <variant...>  (A/B of ab/libfrecsys_hip_<v>.so, built by `make abvar`, against the tree's library: GPU parity tests on each variant, alternating bench lines, FRECSYS_DUAL_PROF phase cycles)
set -o pipefail
OUT=gpurun_out/$1; shift
VS="$*"
mkdir -p $OUT
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
cp $LIB $OUT/base.so.bak
restore() { cp $OUT/base.so.bak $LIB; }
trap restore EXIT
for v in $VS; do
  cp ab/libfrecsys_hip_$v.so $LIB
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py tests/test_dual_gpu.py tests/test_split_gpu.py tests/test_models_gpu.py > $OUT/pytest_$v.log 2>&1; rc=$?
  echo "$v pytest rc=$rc"; tail -2 $OUT/pytest_$v.log
  [ $rc -ne 0 ] && { restore; exit $rc; }
done
summ() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], round(d['ms_per_step'],3))" $1 $2; }
for rep in 1 2 3; do
  for v in base $VS; do
    if [ $v = base ]; then restore; else cp ab/libfrecsys_hip_$v.so $LIB; fi
    for w in ials_ml20m_d256 safer2_ml20m_d256; do
      timeout -k 10 300 python bench.py --allow-env --workload $w --extras= --cpu-seconds 0 --steps 20 --warmup 3 --quiet > $OUT/${w}_${v}_$rep.json 2> $OUT/${w}_${v}_$rep.err || { echo bench failed; tail -5 $OUT/${w}_${v}_$rep.err; restore; exit 5; }
      summ $OUT/${w}_${v}_$rep.json ${w}_${v}_$rep
    done
  done
done
for v in base $VS; do
  if [ $v = base ]; then restore; else cp ab/libfrecsys_hip_$v.so $LIB; fi
  FRECSYS_DUAL_SERIAL=1 FRECSYS_DUAL_PROF=1 timeout -k 10 300 python bench.py --allow-env --workload ials_ml20m_d256 --extras= --cpu-seconds 0 --steps 1 --warmup 1 --quiet > $OUT/prof_$v.json 2> $OUT/prof_$v.err || { echo prof failed; tail -5 $OUT/prof_$v.err; restore; exit 6; }
  echo "== $v"; grep -E "dspace-prof|dual-prof" $OUT/prof_$v.err | head -14
done
restore
rm -f $OUT/base.so.bak
