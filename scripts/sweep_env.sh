#!/bin/bash
# Headline sec/epoch under a few path-selector settings (two runs each).
# Usage: sweep_env.sh <outdir> "<ENV=V ...>" ...   ("-" = defaults)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
shift
mkdir -p $OUT
i=0
for cfg in "$@"; do
  i=$((i+1))
  for rep in 1 2; do
    if [ "$cfg" = "-" ]; then
      timeout -k 10 200 python bench.py --extras= --steps 5 --warmup 2 --cpu-seconds 0 --quiet > $OUT/b_${i}_$rep.json 2> $OUT/b_${i}_$rep.err || exit 2
    else
      timeout -k 10 200 env $cfg python bench.py --extras= --steps 5 --warmup 2 --cpu-seconds 0 --quiet --allow-env > $OUT/b_${i}_$rep.json 2> $OUT/b_${i}_$rep.err || exit 2
    fi
    echo "$cfg run $rep: ms/epoch $(python3 -c "import json; print(round(json.load(open('$OUT/b_${i}_$rep.json'))['ms_per_step'], 3))")"
  done
done
