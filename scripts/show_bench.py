"""Print the headline and per-workload figures of a bench.py JSON line."""
import json
import sys

line = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])


def show(r, name):
    print(f"{name}: value {r['value']:.0f} sec/epoch {r['sec_per_epoch']:.4f} "
          f"roofline {r['roofline']['frac']:.3f} ({r['roofline']['avg_launch_ms']:.3f} ms/launch) "
          f"gather {r['gather_roofline']['frac']:.3f} loss-gather {r['loss_gather_roofline']['frac']:.3f} "
          f"cpu {r['cpu_baseline'] and round(r['cpu_baseline']['value'])}")
    print("   ", {k: round(v, 3) for k, v in r["kernel_ms_per_epoch"].items() if v})


show(line, line["config"]["workload"].split(":")[0])
for k, r in line.get("workloads", {}).items():
    show(r, k)
