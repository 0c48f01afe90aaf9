set -o pipefail
OUT=gpurun_out/r4c
mkdir -p $OUT
fatal() { case $1 in 124|137|134|139|143) return 0;; esac; return 1; }
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_wide_split_gpu.py -k "variants" > $OUT/pytest_var.log 2>&1; rc=$?
tail -3 $OUT/pytest_var.log
fatal $rc && exit $rc
FRECSYS_WIDE_CHOL_RD=3 timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_wide_split_gpu.py -k "parity or weighted_v" > $OUT/pytest_rd3.log 2>&1; rc=$?
tail -3 $OUT/pytest_rd3.log
fatal $rc && exit $rc
for rd in 1 2 3 4; do
  FRECSYS_WIDE_CHOL_RD=$rd FRECSYS_W2_AHEAD=${AH:-1} timeout -k 10 300 python bench.py --allow-env --workload ials_msd_d512 --extras= --cpu-seconds 0 --steps 5 --warmup 2 --quiet > $OUT/ab_rd$rd.json 2> $OUT/ab_rd$rd.err || { echo ab $rd failed; tail -5 $OUT/ab_rd$rd.err; exit 5; }
  python3 -c "import json;d=json.load(open('$OUT/ab_rd$rd.json'));k=d['kernel_ms_per_epoch'];print('rd=$rd', round(d['ms_per_step'],2), {x: round(k[x],2) for x in ('solve_user','solve_item','solve_user.dspace','solve_item.dspace')})"
done
