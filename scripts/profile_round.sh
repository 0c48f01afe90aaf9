#!/bin/bash
# Measurement pass for the round (run on the GPU box through gpurun):
#   1. the default bench line (headline + extra workloads, CPU baselines)
#   2. per workload: rocprofv3 kernel stats of the same command, then the
#      FETCH_SIZE and WRITE_SIZE passes (separate runs, no tracing domains),
#      summarised into profiles/latest_pmc.json by scripts/pmc_summary.py
#   3. serialised streams (FRECSYS_DUAL_SERIAL=1): kernel stats + one SQ pass
#      (MFMA busy, wait/issue stalls) of the headline workload
#   4. scripts/gather_prof.sh: the MSD item half-step's fabric bytes (marker-
#      bracketed FETCH / WRITE passes) and the FETCH_SIZE width calibration,
#      merged into latest_pmc.json (halfstep_item)
# Usage: profile_round.sh <outdir under gpurun_out> [workloads...]
#   SKIP_BENCH=1: no step 1; SKIP_TAIL=1: no steps 3-4 (to split the pass over calls)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
NAME=$1
OUT=gpurun_out/$NAME
shift
WL=${*:-ials_ml20m_d256 safer2_ml20m_d256 ials_msd_d512}
mkdir -p $OUT
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; exit 1; }
  echo "bench ok"
fi
for w in $WL; do
  ARGS="--workload $w --extras= --steps 10 --warmup 1 --cpu-seconds 0 --quiet"
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_$w -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace_$w.log 2>&1 || { echo trace $w failed; exit 2; }
  PARGS="--workload $w --extras= --steps 1 --warmup 1 --cpu-seconds 0 --quiet"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_$w -o run --output-format csv -- python3 bench.py $PARGS > $OUT/fetch_$w.log 2>&1 || { echo fetch $w failed; exit 3; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write_$w -o run --output-format csv -- python3 bench.py $PARGS > $OUT/write_$w.log 2>&1 || { echo write $w failed; exit 4; }
  python3 scripts/pmc_summary.py $w $(ls $OUT/fetch_$w/*counter_collection.csv $OUT/fetch_$w/*/*counter_collection.csv 2>/dev/null | head -1) $(ls $OUT/write_$w/*counter_collection.csv $OUT/write_$w/*/*counter_collection.csv 2>/dev/null | head -1) 2 $OUT/pmc_$w.json $OUT/latest_pmc.json > $OUT/pmc_$w.txt || { echo summary $w failed; exit 5; }
  echo "$w ok"
done
[ -n "$SKIP_TAIL" ] && { echo done; exit 0; }
SARGS="--workload ials_ml20m_d256 --extras= --steps 2 --warmup 1 --cpu-seconds 0 --quiet --allow-env"
FRECSYS_DUAL_SERIAL=1 timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/trace_serial -o run --output-format csv -- python3 bench.py $SARGS > $OUT/trace_serial.log 2>&1 || { echo serial trace failed; exit 6; }
FRECSYS_DUAL_SERIAL=1 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/sq_serial -o run --output-format csv -- python3 bench.py $SARGS > $OUT/sq_serial.log 2>&1 || { echo sq pass failed; exit 7; }
# the gather on a table past the Infinity Cache (MSD item half-step) + the
# FETCH_SIZE calibration of the access widths
./scripts/gather_prof.sh $NAME/gather ials_msd_d512 item || { echo gather prof failed; exit 8; }
python3 scripts/pmc_halfstep.py $OUT/gather/fetch/run_counter_collection.csv $OUT/gather/write/run_counter_collection.csv $OUT/gather/probe.json 2.0 $OUT/gather_msd_item.json $OUT/latest_pmc.json > /dev/null || { echo halfstep summary failed; exit 9; }
echo done
