#!/bin/bash
# Serialised streams (FRECSYS_DUAL_SERIAL=1): the bench line's per-path timers
# (d-space / history-space / basis / rotate per half-step, no CU sharing) and
# rocprofv3 kernel stats of the same command, for each workload.
# Usage: serial_paths.sh <outdir under gpurun_out> <workload...>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for W in "$@"; do
  S=3; [ $W = safer2_2m500k_d1024 ] && S=2; [ $W = ials_ml20m_d256 ] && S=10
  FRECSYS_DUAL_SERIAL=1 timeout -k 10 400 python bench.py --allow-env --workload $W --extras= --cpu-seconds 0 --steps $S --warmup 1 --quiet > $OUT/serial_$W.json 2> $OUT/serial_$W.err || { echo "bench $W failed"; tail -5 $OUT/serial_$W.err; exit 1; }
  python3 -c "
import json,sys
d=json.load(open(sys.argv[1]));k=d['kernel_ms_per_epoch']
print(sys.argv[2], 'ms/step', round(d['ms_per_step'],2))
for s in ('solve_user','solve_item'):
    p=d['paths'][s]
    print(' ', s, ' '.join(f'{n}={k[s+\".\"+n]:.2f}' for n in ('dspace','split','basis','hspace','rotate')), 'dspace_tf', p['dspace_tflops'] and round(p['dspace_tflops'],1), 'hspace_tf', p['hspace_tflops'] and round(p['hspace_tflops'],1))
print('  gramian', round(k['gramian'],2), 'loss', round(k['user_loss'],2))" $OUT/serial_$W.json $W
  FRECSYS_DUAL_SERIAL=1 timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $OUT/trace_$W -o run --output-format csv -- python3 bench.py --allow-env --workload $W --extras= --cpu-seconds 0 --steps $S --warmup 1 --quiet > $OUT/trace_$W.log 2>&1 || { echo "trace $W failed"; tail -5 $OUT/trace_$W.log; exit 2; }
  python3 scripts/kstats.py $OUT/trace_$W/run_kernel_stats.csv $((S + 1)) 30 > $OUT/kstats_serial_$W.txt
  rm -rf $OUT/trace_$W/*kernel_trace.csv
done
