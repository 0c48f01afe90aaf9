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
