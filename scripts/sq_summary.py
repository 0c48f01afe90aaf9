"""Per-kernel SQ counter summary of a rocprofv3 --pmc pass (serialised streams):
MFMA busy share, wave-cycle split (active / issue-stalled / parked), instruction mix.
Units (MI355X_MICROARCH.md): SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_ANY count
quad-cycles per wave; SQ_BUSY_CYCLES and SQ_VALU_MFMA_BUSY_CYCLES count cycles
(MFMA busy summed over the SIMDs); SQ_BUSY_CYCLES is summed over the 32 shader
engines (8 XCDs x 4 SEs: BUSY / 32 = the kernel's duration in cycles, checked
against the dispatch timestamps).  MFMA busy % = MFMA_BUSY / (BUSY/32 x 4 SIMD x CUs).
Usage: sq_summary.py <counter_collection.csv> <n_cu> [out.json]"""
import collections
import csv
import json
import sys

path, ncu = sys.argv[1], int(sys.argv[2])
acc = collections.defaultdict(lambda: collections.defaultdict(float))
launches = collections.defaultdict(set)
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"].replace("frecsys_hip::(anonymous namespace)::", "").split("(")[0]
    acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
    launches[name].add(r["Dispatch_Id"])
out = {}
for name, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CYCLES", 0)):
    busy = c.get("SQ_BUSY_CYCLES", 0.0)
    wave = c.get("SQ_WAVE_CYCLES", 0.0)
    if busy <= 0 or wave <= 0:
        continue
    row = {
        "launches": len(launches[name]),
        "mfma_busy_frac": c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (busy / 32.0 * 4 * ncu),
        "wave_active_frac": c.get("SQ_ACTIVE_INST_ANY", 0.0) / wave,
        "wave_issue_stall_frac": c.get("SQ_WAIT_INST_ANY", 0.0) / wave,
        "wave_parked_frac": c.get("SQ_WAIT_ANY", 0.0) / wave,
        "valu_insts": c.get("SQ_INSTS_VALU", 0.0),
        "lds_insts": c.get("SQ_INSTS_LDS", 0.0),
    }
    out[name] = row
    print(f"{name:34s} n={row['launches']:3d} mfma_busy {row['mfma_busy_frac']:.3f} "
          f"active {row['wave_active_frac']:.2f} issue-stall {row['wave_issue_stall_frac']:.2f} "
          f"parked {row['wave_parked_frac']:.2f}")
if len(sys.argv) > 3:
    json.dump({"source": path, "n_cu": ncu, "kernels": out}, open(sys.argv[3], "w"), indent=1)
