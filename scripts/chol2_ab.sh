# A/B of the wide Cholesky kernels: bit-identity diagnostics, the wide GPU
# tests, and the MSD iALS bench with FRECSYS_WIDE_CHOL2=1 / 0 twice each.
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/chol2_diag.py
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_wide_chol2_gpu.py tests/test_wide_split_gpu.py tests/test_wide_gpu.py > gpurun_out/c2_tests.log 2>&1
tail -3 gpurun_out/c2_tests.log
for v in 1 0 1 0; do
  FRECSYS_WIDE_CHOL2=$v timeout -k 10 200 python bench.py --allow-env --workload ials_msd_d512 --steps 5 --warmup 2 > gpurun_out/c2_b$v.json 2>gpurun_out/c2_b$v.err
  python -c "import json;d=json.load(open('gpurun_out/c2_b$v.json'));print('chol2',$v,d['ms_per_step'])"
done
