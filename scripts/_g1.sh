set -o pipefail
OUT=gpurun_out/r4a
mkdir -p $OUT
fatal() { case $1 in 124|137|134|139|143) return 0;; esac; return 1; }
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_models_gpu.py -k "residual or reg_exp0" > $OUT/pytest_models.log 2>&1; rc=$?
tail -3 $OUT/pytest_models.log
fatal $rc && exit $rc
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_dual_gpu.py tests/test_workload_gpu.py > $OUT/pytest_dw.log 2>&1; rc=$?
tail -3 $OUT/pytest_dw.log
fatal $rc && exit $rc
bash scripts/msd_prof.sh r4a/msd
for v in 1 2; do
  FRECSYS_W2_AHEAD=$v timeout -k 10 300 python bench.py --allow-env --workload ials_msd_d512 --extras= --cpu-seconds 0 --steps 5 --warmup 2 --quiet > gpurun_out/r4a/ab_ah1_$v.json 2> gpurun_out/r4a/ab_ah1_$v.err || { echo ab $v failed; tail -5 gpurun_out/r4a/ab_ah1_$v.err; exit 5; }
  python3 -c "import json;d=json.load(open('gpurun_out/r4a/ab_ah1_$v.json'));k=d['kernel_ms_per_epoch'];print('ahead=$v', round(d['ms_per_step'],2), {x: round(k[x],2) for x in ('solve_user','solve_item','solve_user.dspace','solve_item.dspace','solve_user.hspace','solve_item.hspace')})"
done
