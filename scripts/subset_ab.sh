#!/bin/bash
# Row-subset forward rotation (FRECSYS_ROT_SUBSET): GPU suite, then the
# per-rank epoch at N = 8 of configs 2 and 4 with and without the subsets
# (scripts/rank_share.py), and the N = 1 headline bench.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-subset} && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; tail -2 $O/pytest.log
for wl in ials_ml20m_d256 ials_msd_d512; do
  for sub in 1 0; do
    FRECSYS_ROT_SUBSET=$sub timeout -k 10 300 python3 scripts/rank_share.py $wl 3 8 > $O/rs_${wl}_$sub.jsonl 2> $O/rs_${wl}_$sub.err || { echo rank_share failed; tail -5 $O/rs_${wl}_$sub.err; exit 1; }
    echo "$wl subset=$sub $(tail -1 $O/rs_${wl}_$sub.jsonl)"
  done
done
timeout -k 10 200 python bench.py --extras= --steps 20 --warmup 3 --cpu-seconds 0 > $O/bench.json 2>/dev/null && python3 -c "import json; b=json.load(open('$O/bench.json')); print('bench', round(b['ms_per_step'],3))"
echo done
