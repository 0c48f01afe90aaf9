#!/bin/bash
# A/B of the split-bf16 SYRK tile ownership (FRECSYS_SYRK_SB builds 0 / 1 / 2
# under scripts/micro/sbN/): bit-for-bit d-space outputs (lib_ab_dump.py),
# then the headline bench with each build in place of the in-tree library.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/sb && mkdir -p $O
for v in 0 1 2; do
  timeout -k 10 120 python3 scripts/lib_ab_dump.py scripts/micro/sb$v/libfrecsys_hip.so $O/d$v.npz > $O/dump_$v.log 2>&1 || { echo dump $v failed; tail -5 $O/dump_$v.log; exit 1; }
done
python3 -c "
import numpy as np
a=np.load('$O/d0.npz')
for v in (1, 2):
    b=np.load('$O/d%d.npz' % v); print(v, {k: int((a[k]!=b[k]).sum()) for k in a.files})"
timeout -k 10 300 python -u -m pytest tests/test_split_gpu.py tests/test_parity_gpu.py -q --timeout 60 --timeout-method thread > $O/pytest.log 2>&1; tail -2 $O/pytest.log
for v in 0 1 2 0 1 2; do
  cp scripts/micro/sb$v/libfrecsys_hip.so safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
  timeout -k 10 150 python bench.py --extras= --steps 20 --warmup 3 --cpu-seconds 0 > $O/bench_$v.json 2> /dev/null || { echo bench $v failed; exit 2; }
  python3 -c "import json; b=json.load(open('$O/bench_$v.json')); print('sb$v', round(b['ms_per_step'],3), {k: round(v,3) for k,v in b['kernel_ms_per_epoch'].items() if k in ('solve_user.dspace','solve_item.dspace','solve_item.split')})"
done
for v in 0 2; do
  cp scripts/micro/sb$v/libfrecsys_hip.so safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
  FRECSYS_DUAL_SERIAL=1 timeout -k 10 150 python bench.py --extras= --steps 10 --warmup 2 --cpu-seconds 0 --allow-env > $O/serial_$v.json 2>/dev/null || exit 3
  python3 -c "import json; b=json.load(open('$O/serial_$v.json')); print('serial sb$v', round(b['ms_per_step'],3), {k: round(v,3) for k,v in b['kernel_ms_per_epoch'].items() if k in ('solve_user.dspace','solve_item.dspace','solve_item.split')})"
done
rm -f $O/*.npz
echo done
