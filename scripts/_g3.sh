set -o pipefail
OUT=gpurun_out/r4a
mkdir -p $OUT
fatal() { case $1 in 124|137|134|139|143) return 0;; esac; return 1; }
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_wide_split_gpu.py tests/test_dual_gpu.py tests/test_pp_gpu.py -k "variants or conditioning or sharded" > $OUT/pytest_ah2.log 2>&1; rc=$?
tail -3 $OUT/pytest_ah2.log
fatal $rc && exit $rc
FRECSYS_WIDE_CHOL_RD=2 timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_wide_split_gpu.py -k "parity or weighted_v" > $OUT/pytest_rd2.log 2>&1; rc=$?
tail -3 $OUT/pytest_rd2.log
fatal $rc && exit $rc
bash scripts/msd_prof.sh r4a/msd
for v in 1 2 3 4 5; do
  rd=0; ah=$v; ws=4096; [ $v = 3 ] && { rd=1; ah=2; }; [ $v = 4 ] && { rd=1; ah=2; ws=12288; }; [ $v = 5 ] && { rd=2; ah=2; }
  FRECSYS_WIDE_WS_MB=$ws FRECSYS_WIDE_CHOL_RD=$rd FRECSYS_W2_AHEAD=$ah timeout -k 10 300 python bench.py --allow-env --workload ials_msd_d512 --extras= --cpu-seconds 0 --steps 5 --warmup 2 --quiet > gpurun_out/r4a/ab_ah1_$v.json 2> gpurun_out/r4a/ab_ah1_$v.err || { echo ab $v failed; tail -5 gpurun_out/r4a/ab_ah1_$v.err; exit 5; }
  python3 -c "import json;d=json.load(open('gpurun_out/r4a/ab_ah1_$v.json'));k=d['kernel_ms_per_epoch'];print('ahead=$v', round(d['ms_per_step'],2), {x: round(k[x],2) for x in ('solve_user','solve_item','solve_user.dspace','solve_item.dspace','solve_user.hspace','solve_item.hspace')})"
done
