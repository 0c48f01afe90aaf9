#!/bin/bash
# A/B of the dataflow Cholesky task order (chol.h): the in-tree library
# against scripts/micro/chol0/ (the previous order) -- bit-for-bit outputs on
# both paths (lib_ab_dump.py), then the headline bench alternating, then
# serialised.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-cholab} && mkdir -p $O
cp safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so $O/new.so
for d in 0 1; do
  for v in new chol0; do
    L=$O/new.so; [ $v = chol0 ] && L=scripts/micro/chol0/libfrecsys_hip.so
    FRECSYS_DUAL=$d timeout -k 10 120 python3 scripts/lib_ab_dump.py $L $O/d_${v}_$d.npz > $O/dump_${v}_$d.log 2>&1 || { echo dump $v $d failed; tail -5 $O/dump_${v}_$d.log; exit 1; }
  done
  python3 -c "
import numpy as np
a=np.load('$O/d_new_$d.npz'); b=np.load('$O/d_chol0_$d.npz'); print('dual=$d', {k: int((a[k]!=b[k]).sum()) for k in a.files})"
done
for v in new chol0 new chol0; do
  L=$O/new.so; [ $v = chol0 ] && L=scripts/micro/chol0/libfrecsys_hip.so
  cp $L safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
  timeout -k 10 150 python bench.py --extras= --steps 20 --warmup 3 --cpu-seconds 0 > $O/bench_$v.json 2>/dev/null || { echo bench failed; exit 2; }
  python3 -c "import json; b=json.load(open('$O/bench_$v.json')); k=b['kernel_ms_per_epoch']; print('$v', round(b['ms_per_step'],3), {x: round(k[x],3) for x in ('solve_user.dspace','solve_item.dspace','solve_user.hspace','solve_item.hspace')})"
done
for v in new chol0; do
  L=$O/new.so; [ $v = chol0 ] && L=scripts/micro/chol0/libfrecsys_hip.so
  cp $L safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
  FRECSYS_DUAL_SERIAL=1 timeout -k 10 150 python bench.py --extras= --steps 10 --warmup 2 --cpu-seconds 0 --allow-env > $O/serial_$v.json 2>/dev/null || exit 3
  python3 -c "import json; b=json.load(open('$O/serial_$v.json')); k=b['kernel_ms_per_epoch']; print('serial $v', round(b['ms_per_step'],3), {x: round(k[x],3) for x in ('solve_user.dspace','solve_item.dspace','solve_user.hspace','solve_item.hspace')})"
done
cp $O/new.so safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
rm -f $O/*.npz $O/new.so
echo done
