"""Print ms_per_step and the top kernels (ms per epoch) of an ab_env.sh run."""
import csv, glob, json, os, sys
out = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
for b in sorted(glob.glob(os.path.join(out, "bench_*.json"))):
    i = b.rsplit("_", 1)[1].split(".")[0]
    try:
        print(f"variant {i}: ms/epoch {json.load(open(b))['ms_per_step']:.3f}")
    except Exception as e:
        print(f"variant {i}: {e}")
    st = os.path.join(out, f"trace_{i}", "run_kernel_stats.csv")
    if os.path.exists(st):
        rows = list(csv.reader(open(st)))[1:]
        for r in rows[:n]:
            nm = r[0].replace("frecsys_hip::(anonymous namespace)::", "").replace("void ", "")
            print(f"   {nm[:58]:58s} {float(r[2]) / 3 / 1e6:7.3f}")
