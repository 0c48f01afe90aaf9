#!/usr/bin/env python3
"""Timeline of the last epoch in a rocprofv3 --kernel-trace CSV (one process,
e.g. scripts/rank_share.py <workload> <steps> <N> <rank>): every kernel's
start / end relative to the epoch's first kernel, grouped by the epoch phases
(the Gramian launches delimit them), plus the busy time of the union of all
kernels and the idle gaps.

Usage: timeline_summary.py <kernel_trace.csv> <marker> [out.json]
  marker: substring of the kernel that closes an epoch (the user loss:
  loss_gather); the last epoch = the kernels after the second-to-last
  marker up to the last one."""
import csv
import json
import re
import sys


def short(name):
    name = re.sub(r"frecsys_hip::\(anonymous namespace\)::", "", name)
    name = re.sub(r"\(frecsys_hip::[A-Za-z]+\)", "", name)
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "")
    if name.startswith("_ZN11frecsys_hip12_GLOBAL__N_1"):
        m = re.match(r"_ZN11frecsys_hip12_GLOBAL__N_1\d+([a-z_]+)ILi(\d+)E", name)
        if m:
            name = f"{m.group(1)}<{m.group(2)}>"
    return name


def main():
    path, marker = sys.argv[1], sys.argv[2]
    rows = list(csv.DictReader(open(path)))
    ks = sorted(({"name": short(r["Kernel_Name"]), "s": int(r["Start_Timestamp"]),
                  "e": int(r["End_Timestamp"])} for r in rows), key=lambda k: k["s"])
    ends = [i for i, k in enumerate(ks) if marker in k["name"]]
    ep = ks[ends[-2] + 1:ends[-1] + 1]
    t0 = ep[0]["s"]
    busy, cur_s, cur_e = 0, None, None
    for k in ep:
        if cur_e is None or k["s"] > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = k["s"], k["e"]
        else:
            cur_e = max(cur_e, k["e"])
    busy += cur_e - cur_s
    span = max(k["e"] for k in ep) - t0
    out = {"epoch_span_us": span / 1e3, "busy_us": busy / 1e3,
           "kernels": [{"name": k["name"], "start_us": round((k["s"] - t0) / 1e3, 1),
                        "dur_us": round((k["e"] - k["s"]) / 1e3, 1)} for k in ep]}
    for k in out["kernels"]:
        print(f'{k["start_us"]:9.1f} {k["dur_us"]:8.1f}  {k["name"]}')
    print(f"epoch span {span / 1e3:.1f} us, union busy {busy / 1e3:.1f} us")
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
