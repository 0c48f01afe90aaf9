#!/bin/bash
# SQ stall breakdown of one bench.py workload's kernels (one --pmc pass per
# counter set, no tracing domains), summarised by sq_summary.py.
# Usage: pmc_sq_w.sh <outdir> <workload>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
W=$2
mkdir -p $OUT
FRECSYS_DUAL_SERIAL=1 timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/pmc -o run --output-format csv -- python3 bench.py --workload $W --extras= --allow-env --steps 1 --warmup 0 --cpu-seconds 0 --quiet > $OUT/pmc.log 2>&1 || exit 3
F=$(ls $OUT/pmc/*counter_collection.csv $OUT/pmc/*/*counter_collection.csv 2>/dev/null | head -1)
python3 scripts/sq_summary.py $F 256 $OUT/sq.json > /dev/null && python3 -c "
import json; d=json.load(open('$OUT/sq.json'))
for k,v in list(d['kernels'].items())[:8]: print(k[:40], {a:(round(b,3) if isinstance(b,float) else b) for a,b in v.items()})
"
