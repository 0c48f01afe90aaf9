# Round-end check on one GPU box (call 1 of 2): the whole -m gpu suite,
# smoke(), the default bench line.  Usage: final_r04.sh <outdir under gpurun_out>
set -o pipefail
OUT=gpurun_out/${1:-final_r04}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
case $rc in 124|137|134|139|143) exit $rc;; esac
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 2; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 3; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['ms_per_step'], d['value'], d['roofline']['frac'], {k: v['ms_per_step'] for k, v in d.get('workloads', {}).items()})"
exit $rc
