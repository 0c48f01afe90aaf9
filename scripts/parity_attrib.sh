#!/bin/bash
# Attribution of the wide-dim parity maxima (run on the GPU box): the
# l2_reg_exp = 0 cases and the trained-spectrum half-steps under
#   base       the shipped library
#   cholbasis0 FRECSYS_CHOL_BASIS=0 (tridiagonal basis for l2_reg_exp = 0)
#   syrkf32    FRECSYS_SYRK_F32=1 (fp32 MFMA products in the history-space
#              S assembly and the d <= 256 SYRK instead of split-bf16)
#   x6off      ab/libfrecsys_hip_x6off.so (make abvar ABDEF=-DFRECSYS_CHOL_X6=0
#              ABNAME=x6off): fp32 TRSM / trailing products in the LDS Cholesky
# each into gpurun_out/<out>/report_<variant>.jsonl (tests' PARITY_REPORT).
# Usage: parity_attrib.sh <outdir under gpurun_out> <variant...>
set -o pipefail
OUT=gpurun_out/$1
shift
mkdir -p $OUT
LIB=safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
cp $LIB $OUT/base.so.bak
restore() { cp $OUT/base.so.bak $LIB; }
trap restore EXIT
ALL="tests/test_reg_exp0_gpu.py tests/test_dual_gpu.py::test_wide_trained_spectrum_half_step tests/test_models_gpu.py::test_ials_reg_exp0_trajectory_matches_oracle"
TRAJ="tests/test_models_gpu.py::test_ials_reg_exp0_trajectory_matches_oracle"
run() {  # <variant> <tests> [env assignments...]
  local v=$1 SEL=$2; shift 2
  env PARITY_REPORT=$PWD/$OUT/report_$v.jsonl "$@" timeout -k 10 900 python -u -m pytest -q -s \
    --timeout 300 --timeout-method thread $SEL > $OUT/pytest_$v.log 2>&1
  local rc=$?
  echo "$v rc=$rc"; tail -2 $OUT/pytest_$v.log
  # a failing assertion is data here; a crash / timeout ends the script
  [ $rc -le 1 ] || exit $rc
}
for v in "$@"; do
  case $v in
    base) run base "$ALL" ;;
    cholbasis0) run cholbasis0 "$TRAJ" FRECSYS_CHOL_BASIS=0 ;;
    syrkf32) run syrkf32 "$ALL" FRECSYS_SYRK_F32=1 ;;
    x6off) cp ab/libfrecsys_hip_x6off.so $LIB && run x6off "$ALL"; restore ;;
  esac
done
echo done
