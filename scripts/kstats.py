"""Per-epoch kernel time table of a rocprofv3 kernel_stats.csv.
Usage: kstats.py <run_kernel_stats.csv> <epochs in the run> [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ep = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 24
tot = 0.0
for r in rows:
    tot += float(r["TotalDurationNs"])
for r in rows[:top]:
    short = r["Name"].replace("frecsys_hip::(anonymous namespace)::", "").removeprefix("void ")[:58]
    print(f"{short:60s} calls {r['Calls']:>5} avg_us {float(r['AverageNs']) / 1e3:9.1f} "
          f"ms/epoch {float(r['TotalDurationNs']) / 1e6 / ep:8.3f}")
print(f"total kernel ms/epoch {tot / 1e6 / ep:.3f}")
