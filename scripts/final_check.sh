# Round-end check on one GPU box: the whole -m gpu suite, smoke(), the default bench line.
set -o pipefail
OUT=gpurun_out/${1:-final2}
mkdir -p $OUT
timeout -k 10 780 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 2; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 3; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['ms_per_step'], d['value'], [(k, round(e['ms_per_step'], 2)) for k, e in d.get('workloads', {}).items()])"
