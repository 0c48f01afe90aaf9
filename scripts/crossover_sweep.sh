#!/bin/bash
# Per-side crossover sweep of the headline epoch (FRECSYS_DUAL_MAX_H_USER /
# _ITEM: longest h_eff on the history-space path of each side).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-xover} && mkdir -p $O
for cfg in "224 224" "224 256" "224 192" "256 224" "192 224" "224 224"; do
  set -- $cfg
  FRECSYS_DUAL_MAX_H_USER=$1 FRECSYS_DUAL_MAX_H_ITEM=$2 timeout -k 10 150 python bench.py --extras= --steps 20 --warmup 3 --cpu-seconds 0 --allow-env > $O/b_$1_$2.json 2>/dev/null || exit 1
  python3 -c "import json; b=json.load(open('$O/b_$1_$2.json')); k=b['kernel_ms_per_epoch']; print('user $1 item $2', round(b['ms_per_step'],3), {x: round(k[x],2) for x in ('solve_user','solve_item','solve_user.dspace','solve_user.hspace','solve_item.dspace','solve_item.hspace')})"
done
