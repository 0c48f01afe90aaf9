#!/bin/bash
# Timing ablation (wrong numbers): the library built with FRECSYS_CHEAP_SPLIT
# (split3 keeps only the hi piece) swapped in, serialised kernel stats of the
# headline and the MSD workload -- the upper bound of what removing the
# split's VALU work from the staging would save.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
[ "$2" = base ] || cp ab/cs/libfrecsys_hip.so safer2-recommender_amd/frecsys_hip/libfrecsys_hip.so
for w in ials_ml20m_d256 ials_msd_d512; do
  FRECSYS_DUAL_SERIAL=1 timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/cs_$w -o run --output-format csv -- python3 bench.py --workload $w --extras= --steps 2 --warmup 1 --cpu-seconds 0 --quiet --allow-env > $OUT/cs_$w.log 2>&1 || { echo fail $w; tail -5 $OUT/cs_$w.log; exit 3; }
  python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/cs_$w/run_kernel_stats.csv')))[:10]: print('$w', '%-60s %8.3f'%(r['Name'][:60], float(r['TotalDurationNs'])/3e6))
"
done
