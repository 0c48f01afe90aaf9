"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of one bench.py
workload into per-launch fabric traffic (bytes) per kernel, and the traffic
of the workload's roofline kernel per d-space call (the unit bench.py's
`roofline.achieved` is per).

gfx950 correction (/opt/skills/guides/MI355X_MICROARCH.md, HBM section):
FETCH_SIZE (KiB, = TCC_EA0_RDREQ x 64 B) reports half the bytes of 16-B/lane
streaming reads -> x2; WRITE_SIZE as is.  The solve kernels gather 4-B/lane
(one float per lane, 64 lanes = one 256-B row segment): that width is not
calibrated by the guide, so both the raw and the x2 figures are kept.

Usage: pmc_summary.py <workload> <fetch.csv> <write.csv> <epochs> <out.json> [<merge.json>]
  epochs: Train() epochs the pass ran (warmup + steps); the d-space solve runs
  once per half-step, 2 per epoch.
scripts/micro/fetch_cal.hip measured the x2 for this code's widths as well:
4-B/lane reads of 256 contiguous bytes and 4-B/lane gathers of 2-KB rows of a
1.2 GB table both report 0.50-0.51 of the bytes (profiles/r03/fetch_cal.json).
"""
import csv
import json
import os
import sys


def per_kernel(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]) * 1024.0)
    return out


def loss_kernel(name):
    """The gather kernels of ComputeUserLoss (the u^T G u part runs as a
    rotation / quad kernel and is not a gather)."""
    return "loss_gather" in name


def dominant(name, workload):
    if "d512" in workload or "d1024" in workload:
        # the batched d-space call: the pre-split table, slab SYRK, entity
        # SYRK and Cholesky launches (wide_syrk2: FRECSYS_WIDE_PRESPLIT=0)
        return any(k in name for k in ("wide_presplit_kernel", "wide_syrk3_kernel<1",
                                       "wide_syrk3_kernel<2", "wide_syrk2_kernel<1>",
                                       "wide_syrk2_kernel<2>", "wide_chol_kernel",
                                       "wide_chol2_kernel"))
    return "solve_tiled_kernel<8, false" in name


def main():
    workload, fpath, wpath, epochs, out = sys.argv[1:6]
    merge = sys.argv[6] if len(sys.argv) > 6 else None
    calls = 2 * int(epochs)
    fetch = per_kernel(fpath, "FETCH_SIZE")
    write = per_kernel(wpath, "WRITE_SIZE")
    summary = {"workload": workload, "epochs": int(epochs),
               "correction": "FETCH_SIZE x2 (gfx950: 0.50 of the bytes for 16-B/lane reads per "
                             "MI355X_MICROARCH.md, and for this code's 4-B/lane reads and row "
                             "gathers per scripts/micro/fetch_cal.hip), WRITE_SIZE x1",
               "kernels": {}}
    dom_f = dom_f_raw = dom_w = 0.0
    loss_b, loss_n = 0.0, 0
    for name in sorted(set(fetch) | set(write)):
        f = fetch.get(name, [])
        w = write.get(name, [])
        summary["kernels"][name] = {
            "launches": max(len(f), len(w)),
            "fetch_bytes_per_launch_raw": sum(f) / max(1, len(f)),
            "fetch_bytes_per_launch": 2.0 * sum(f) / max(1, len(f)),
            "write_bytes_per_launch": sum(w) / max(1, len(w)),
        }
        if dominant(name, workload):
            dom_f += 2.0 * sum(f)
            dom_f_raw += sum(f)
            dom_w += sum(w)
        if loss_kernel(name):
            loss_b += 2.0 * sum(f) + sum(w)
            loss_n = max(loss_n, len(f), len(w))
    summary["dominant_traffic_bytes"] = (dom_f + dom_w) / calls
    summary["dominant_traffic_bytes_raw_fetch"] = (dom_f_raw + dom_w) / calls
    summary["loss_fabric_bytes_per_pass"] = loss_b / max(loss_n, 1)
    json.dump(summary, open(out, "w"), indent=1)
    if merge:
        js = json.load(open(merge)) if os.path.exists(merge) else {}
        w = js.setdefault("workloads", {}).setdefault(workload, {})
        w.update({
            "dominant_traffic_bytes": summary["dominant_traffic_bytes"],
            "dominant_traffic_bytes_raw_fetch": summary["dominant_traffic_bytes_raw_fetch"],
            "loss_fabric_bytes_per_pass": summary["loss_fabric_bytes_per_pass"]})
        js["source"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py --workload <w> "
                        "(profiles/<round>/pmc_<w>.json): fabric-side bytes (L2 misses incl. "
                        "Infinity-Cache hits) of the roofline kernel per d-space call, FETCH x2")
        json.dump(js, open(merge, "w"), indent=1)
    print(json.dumps({k: {"fetch_GB": round(v["fetch_bytes_per_launch"] / 1e9, 4),
                          "write_GB": round(v["write_bytes_per_launch"] / 1e9, 4),
                          "launches": v["launches"]}
                      for k, v in summary["kernels"].items()}, indent=1))


if __name__ == "__main__":
    main()
