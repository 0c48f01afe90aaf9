# N = 8 per-rank epoch of config 2 (scripts/rank_share.py) against the
# long-history slab size at Dp <= 256 (FRECSYS_SPLIT_ROWS, default 4096)
set -o pipefail
OUT=gpurun_out/r4f
mkdir -p $OUT
for s in 4096 2048 1024; do
  FRECSYS_SPLIT_ROWS=$s timeout -k 10 240 python scripts/rank_share.py ials_ml20m_d256 5 8 > $OUT/rs_split$s.jsonl 2> $OUT/rs_split$s.err || { echo rs $s failed; tail -5 $OUT/rs_split$s.err; exit 1; }
  echo "split_rows=$s $(tail -1 $OUT/rs_split$s.jsonl)"
done
for s in 2048 1024; do
  FRECSYS_SPLIT_ROWS=$s timeout -k 10 300 python bench.py --allow-env --workload ials_ml20m_d256 --extras= --cpu-seconds 0 --steps 10 --warmup 2 --quiet > $OUT/ml20_split$s.json 2> $OUT/ml20_split$s.err || { echo bench $s failed; exit 2; }
  python3 -c "import json;d=json.load(open('$OUT/ml20_split$s.json'));print('N=1 split $s', round(d['ms_per_step'],2))"
done
