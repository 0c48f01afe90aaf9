"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch
HBM traffic (bytes) per kernel, with the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB, = TCC_EA0_RDREQ
x 64 B) reads half the bytes of wide coalesced streams -> x2; WRITE_SIZE is
taken as is.  Usage: pmc_summary.py <fetch.csv> <write.csv> <out.json>"""
import csv
import json
import sys


def per_kernel(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        out.setdefault(name, []).append(float(r["Counter_Value"]) * 1024.0)
    return out


fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
write = per_kernel(sys.argv[2], "WRITE_SIZE")
summary = {"correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), WRITE_SIZE x1; bytes per launch",
           "kernels": {}}
for name in sorted(set(fetch) | set(write)):
    f = fetch.get(name, [])
    w = write.get(name, [])
    summary["kernels"][name] = {
        "launches": max(len(f), len(w)),
        "fetch_bytes_per_launch_raw": f,
        "fetch_bytes_per_launch": [2.0 * x for x in f],
        "write_bytes_per_launch": w,
    }
# the d-space solve (roofline kernel): launches alternate user, item in
# every bench epoch (warmup included); averaged over all launches
for name, v in summary["kernels"].items():
    if "solve_tiled_kernel<8, false" in name:  # <8, false> / <8, false, BF>
        tot = [a + b for a, b in zip(v["fetch_bytes_per_launch"], v["write_bytes_per_launch"])]
        summary["dspace_traffic_bytes"] = sum(tot) / max(1, len(tot))
        summary["dspace_user_traffic_bytes"] = sum(tot[0::2]) / max(1, len(tot[0::2]))
        summary["dspace_item_traffic_bytes"] = sum(tot[1::2]) / max(1, len(tot[1::2]))
json.dump(summary, open(sys.argv[3], "w"), indent=1)
print(json.dumps({k: {"fetch_GB": [round(x / 1e9, 3) for x in v["fetch_bytes_per_launch"]],
                      "write_GB": [round(x / 1e9, 3) for x in v["write_bytes_per_launch"]]}
                  for k, v in summary["kernels"].items()
                  if "solve" in k or "loss" in k or "dual" in k}, indent=1))
