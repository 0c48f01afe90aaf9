#!/bin/bash
# Per-side crossover sweep of one workload's epoch (FRECSYS_DUAL_MAX_H_USER /
# _ITEM: longest h_eff on the history-space path of each side).
# Usage: crossover_sweep.sh <outdir> [workload] ["u i" pairs...]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-xover} && mkdir -p $O
W=${2:-ials_ml20m_d256}
if [ $# -ge 2 ]; then shift 2; else shift $#; fi
CFGS=("$@")
[ ${#CFGS[@]} -eq 0 ] && CFGS=("224 224" "224 256" "224 192" "256 224" "192 224" "224 224")
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  FRECSYS_DUAL_MAX_H_USER=$1 FRECSYS_DUAL_MAX_H_ITEM=$2 timeout -k 10 150 python bench.py --workload $W --extras= --steps 20 --warmup 3 --cpu-seconds 0 --allow-env > $O/b_$1_$2.json 2>/dev/null || exit 1
  python3 -c "import json; b=json.load(open('$O/b_$1_$2.json')); k=b['kernel_ms_per_epoch']; print('$W user $1 item $2', round(b['ms_per_step'],3), {x: round(k.get(x, 0),2) for x in ('solve_user','solve_item','solve_user.dspace','solve_user.hspace','solve_item.dspace','solve_item.hspace')})"
done
