# N = 8 per-rank epoch of config 2 (scripts/rank_share.py): the item side's
# history-space threshold swept (0 = every item in d space: no basis of G_U
# on the critical path)
set -o pipefail
OUT=gpurun_out/r4b
mkdir -p $OUT
for t in 224 128 0; do
  FRECSYS_DUAL_MAX_H_ITEM=$t timeout -k 10 240 python scripts/rank_share.py ials_ml20m_d256 5 8 > $OUT/rs_item$t.jsonl 2> $OUT/rs_item$t.err || { echo rs $t failed; tail -5 $OUT/rs_item$t.err; exit 1; }
  echo "item_max_h=$t $(tail -1 $OUT/rs_item$t.jsonl)"
done
