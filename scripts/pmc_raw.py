"""Raw per-kernel counter sums of a rocprofv3 --pmc pass (counter_collection.csv),
for the kernels whose names contain any of the given substrings.
Usage: pmc_raw.py <counter_collection.csv> [substring ...]"""
import collections
import csv
import sys

path, keys = sys.argv[1], sys.argv[2:]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
launches = collections.defaultdict(set)
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"].split("(anonymous namespace)::")[-1].split("(")[0]
    if keys and not any(k in name for k in keys):
        continue
    acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
    launches[name].add(r["Dispatch_Id"])
for name, c in acc.items():
    print(f"{name}  launches {len(launches[name])}")
    for k in sorted(c):
        print(f"   {k:32s} {c[k]:.4e}")
    w = c.get("SQ_WAVE_CYCLES")
    if w:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if k in c:
                print(f"   {k + ' / WAVE_CYCLES':32s} {c[k] / w:.3f}")
    if "SQ_LDS_IDX_ACTIVE" in c and "SQ_LDS_BANK_CONFLICT" in c:
        print(f"   {'bank conflict / LDS active':32s} {c['SQ_LDS_BANK_CONFLICT'] / max(c['SQ_LDS_IDX_ACTIVE'], 1):.3f}")
    if "SQ_BUSY_CYCLES" in c and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
        print(f"   {'mfma busy frac (256 CU)':32s} {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (c['SQ_BUSY_CYCLES'] / 32 * 4 * 256):.3f}")
