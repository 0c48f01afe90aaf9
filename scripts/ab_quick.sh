#!/bin/bash
# A/B of the headline epoch: rank_share N = 1 (config 2) and bench, twice each,
# plus the history-space tests (bit-for-bit eager / oracle parity).
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dual_gpu.py tests/test_eager_gpu.py tests/test_parity_gpu.py tests/test_stats_gpu.py tests/test_models_gpu.py tests/test_sharded_gpu.py > $OUT/pytest.log 2>&1 || { echo pytest failed; tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --extras= --cpu-seconds 0 > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { echo bench failed; exit 2; }
  python3 -c "import json; b=json.loads(open('$OUT/bench_$i.json').read().strip().splitlines()[-1]); print('ms/epoch', round(b['ms_per_step'],3), {k: round(v,3) for k,v in b['kernel_ms_per_epoch'].items() if k in ('solve_user','solve_item','solve_user.hspace','solve_item.hspace')})"
done
FRECSYS_DUAL_SERIAL=1 timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/serial -o run --output-format csv -- python3 bench.py --workload ials_ml20m_d256 --extras= --steps 2 --warmup 1 --cpu-seconds 0 --quiet --allow-env > $OUT/serial.log 2>&1 || { echo serial failed; exit 3; }
python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/serial/run_kernel_stats.csv')))[:12]: print('%-60s %7.3f'%(r['Name'][:60], float(r['TotalDurationNs'])/3e6))
"
