# Fabric bytes (FETCH_SIZE) and kernel time of the wide Cholesky, one-panel
# (FRECSYS_WIDE_CHOL2=0) vs two-panel (=1), on the MSD iALS bench (2 steps).
set -e
OUT=gpurun_out/c2pmc
mkdir -p $OUT
for v in 0 1; do
  FRECSYS_WIDE_CHOL2=$v timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/f$v -o run --output-format csv -- python3 bench.py --workload ials_msd_d512 --extras= --steps 2 --warmup 1 --cpu-seconds 0 --quiet --allow-env > $OUT/f$v.log 2>&1 || { echo fetch $v failed; exit 3; }
  FRECSYS_WIDE_CHOL2=$v timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $OUT/t$v -o run --output-format csv -- python3 bench.py --workload ials_msd_d512 --extras= --steps 2 --warmup 1 --cpu-seconds 0 --quiet --allow-env > $OUT/t$v.log 2>&1 || { echo trace $v failed; exit 4; }
done
python3 - <<'PY'
import csv, glob, collections
for v in (0, 1):
    f = glob.glob(f'gpurun_out/c2pmc/f{v}/**/*counter_collection.csv', recursive=True)[0]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        if 'wide_chol' in k:
            agg[k.split('(')[0][-40:]][0] += 1
            agg[k.split('(')[0][-40:]][1] += float(r['Counter_Value'])
    for k, (n, b) in agg.items():
        print(f'chol2={v} {k}: {n} launches, FETCH_SIZE x2 = {2 * b * 1024 / 1e9:.2f} GB')
    s = glob.glob(f'gpurun_out/c2pmc/t{v}/**/*kernel_stats.csv', recursive=True)[0]
    for r in csv.DictReader(open(s)):
        if 'wide_chol' in r['Name']:
            print(f'chol2={v} {r["Name"][:60]}: calls {r["Calls"]} total {float(r["TotalDurationNs"])/1e6:.2f} ms avg {float(r["AverageNs"])/1e3:.1f} us')
PY
