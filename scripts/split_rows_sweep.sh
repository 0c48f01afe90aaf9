#!/bin/bash
# Headline epoch vs the long-history split slab size (FRECSYS_SPLIT_ROWS), N = 1
# and the per-rank epoch at N = 8 (config 2).
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
for r in 4096 6144 8192; do
  for i in 1 2; do
    FRECSYS_SPLIT_ROWS=$r timeout -k 10 200 python bench.py --steps 20 --warmup 5 --extras= --cpu-seconds 0 --allow-env > $OUT/b_${r}_$i.json 2>/dev/null || exit 1
    python3 -c "import json; b=json.loads(open('$OUT/b_${r}_$i.json').read().strip().splitlines()[-1]); print('split $r', round(b['ms_per_step'],3))"
  done
  FRECSYS_SPLIT_ROWS=$r timeout -k 10 200 python scripts/rank_share.py ials_ml20m_d256 5 8 > $OUT/n8_$r.jsonl || exit 2
  echo "n8 $r $(tail -1 $OUT/n8_$r.jsonl)"
done
