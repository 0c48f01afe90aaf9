#!/bin/bash
# MSD (config 4, d = 512) kernel profile with the streams serialised:
# rocprofv3 kernel stats, then one SQ counter pass (scripts/sq_summary.py).
# Usage: msd_prof.sh <outdir under gpurun_out>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
mkdir -p $OUT
FRECSYS_DUAL_SERIAL=1 timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --workload ials_msd_d512 --extras= --cpu-seconds 0 --allow-env --steps 2 --warmup 1 --quiet > $OUT/trace.log 2>&1 || { echo trace failed; tail -5 $OUT/trace.log; exit 1; }
python3 scripts/kstats.py $OUT/trace/run_kernel_stats.csv 3 | tee $OUT/kstats.txt
FRECSYS_DUAL_SERIAL=1 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/pmc -o run --output-format csv -- python3 bench.py --workload ials_msd_d512 --extras= --cpu-seconds 0 --allow-env --steps 1 --warmup 1 --quiet > $OUT/pmc.log 2>&1 || { echo pmc failed; tail -5 $OUT/pmc.log; exit 2; }
python3 scripts/sq_summary.py $OUT/pmc/run_counter_collection.csv 256 $OUT/sq.json | tee $OUT/sq.txt
