#!/usr/bin/env python3
"""Fabric traffic of the half-steps between the two marker dispatches of
scripts/halfstep_probe.py, from rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE
passes (counter_collection.csv), per half-step.

FETCH_SIZE is scaled by the factor measured for the access width by
scripts/micro/fetch_cal.hip (argument; MI355X_MICROARCH.md: x2 for 16-B/lane
streaming reads); WRITE_SIZE as is.  FETCH_SIZE / WRITE_SIZE count the L2's
memory-side requests, Infinity-Cache hits included: fabric bytes, an upper
bound of the HBM bytes.

Usage: pmc_halfstep.py <fetch.csv> <write.csv> <probe.json> <fetch_factor> [out.json [merge.json]]
  merge.json (profiles/latest_pmc.json): the fabric bytes per half-step go to
  workloads.<w>.halfstep_<side> for bench.py."""
import csv
import json
import sys


def between_markers(path, counter):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    marks = [i for i, r in enumerate(rows) if "debug_diag_kernel" in r["Kernel_Name"]]
    assert len(marks) >= 2, "markers not found"
    per = {}
    for r in rows[marks[0] + 1:marks[-1]]:
        if r["Counter_Name"] != counter:
            continue
        per.setdefault(r["Kernel_Name"], 0.0)
        per[r["Kernel_Name"]] += float(r["Counter_Value"]) * 1024.0
    return per


def main():
    fpath, wpath, ppath, factor = sys.argv[1], sys.argv[2], sys.argv[3], float(sys.argv[4])
    probe = json.loads(open(ppath).read().strip().splitlines()[-1])
    reps = probe["reps"]
    fetch = between_markers(fpath, "FETCH_SIZE")
    write = between_markers(wpath, "WRITE_SIZE")
    f = sum(fetch.values()) / reps
    w = sum(write.values()) / reps
    fabric = f * factor + w
    ms = probe["halfstep_ms"]
    out = {"probe": probe, "fetch_factor": factor,
           "fetch_bytes_raw": f, "write_bytes": w, "fabric_bytes": fabric,
           "fabric_gbs": fabric / (ms * 1e-3) / 1e9,
           "algorithmic_gbs": probe["algorithmic_gather_bytes"] / (ms * 1e-3) / 1e9,
           "kernels": {k: {"fetch_raw": v / reps, "write": write.get(k, 0.0) / reps}
                       for k, v in sorted(fetch.items(), key=lambda kv: -kv[1])}}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 5:
        json.dump(out, open(sys.argv[5], "w"), indent=1)
    if len(sys.argv) > 6:
        import os
        m = sys.argv[6]
        js = json.load(open(m)) if os.path.exists(m) else {}
        w = js.setdefault("workloads", {}).setdefault(probe["workload"], {})
        w["halfstep_" + probe["side"]] = {
            "fabric_bytes": fabric, "fetch_factor": factor, "halfstep_ms_probe": ms,
            "algorithmic_gather_bytes": probe["algorithmic_gather_bytes"],
            "gathered_table_bytes": probe["gathered_table_bytes"]}
        json.dump(js, open(m, "w"), indent=1)


if __name__ == "__main__":
    main()
