#!/usr/bin/env python3
"""Per-rank epoch time of the sharded iALS epoch at N = 1, 2, 4, 8, measured on
ONE GPU: a context joins rank r of N with no communicator (external exchange,
include/frecsys_hip.h frecsys_comm_init with id NULL), so it computes exactly
its shard of every half-step -- partial Gramian, own users / items, forward
rotation of the whole other side, loss of its own users -- and skips only the
RCCL exchange.  max over ranks of that time + the modelled exchange is the
N-GPU epoch; the gap to T(1)/N is the replicated work.

Usage: rank_share.py [workload] [steps] [N [rank]]   (workload as bench.py; iALS
only; with N: every rank of that N only; with N rank: that one rank only, e.g. under rocprofv3 --kernel-trace for
scripts/timeline_summary.py)
Prints one JSON line per (N, rank) and a summary line.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "safer2-recommender_amd"))
sys.path.insert(0, ROOT)

import frecsys_hip as fh  # noqa: E402
from frecsys_hip.data import SHAPES, synthetic  # noqa: E402
from bench import WORKLOADS  # noqa: E402

NAMES = ["solve_user", "solve_item", "gramian", "user_loss"]
NAMES += [f"{s}.{p}" for s in ("solve_user", "solve_item")
          for p in ("dspace", "split", "basis", "hspace", "rotate")]


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "ials_ml20m_d256"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    only = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else None
    only_n = int(sys.argv[3]) if len(sys.argv) == 4 else None
    spec = WORKLOADS[wl]
    assert spec["model"] == "ials", "iALS workloads only"
    f = spec["flags"]
    up, uc, ip, ic = synthetic(SHAPES[spec["shape"]])
    nu, ni = len(up) - 1, len(ip) - 1
    summary = {}
    for N in ((only[0],) if only else ((only_n,) if only_n else (1, 2, 4, 8))):
        per_rank = []
        for r in ((only[1],) if only else range(N)):
            ctx = fh.Context(spec["dim"], nu, ni)
            ctx.load_csr(fh.SIDE_USER, up, uc)
            ctx.load_csr(fh.SIDE_ITEM, ip, ic)
            if N > 1:
                ctx.comm_init(N, r, None)
            ctx.init_embeddings(1, 0.1)

            def epoch():
                ctx.gramian(fh.SIDE_ITEM, fetch=False)
                ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, f["l2_reg"], f["uobs_weight"],
                               reg_exp=f["l2_reg_exp"])
                ctx.gramian(fh.SIDE_USER, fetch=False)
                ctx.solve_side(fh.SIDE_ITEM, fh.KIND_IALS, f["l2_reg"], f["uobs_weight"],
                               reg_exp=f["l2_reg_exp"])
                ctx.gramian(fh.SIDE_ITEM, fetch=False)
                ctx.user_loss(fh.SIDE_USER, f["uobs_weight"], False, fetch=False)

            epoch()
            ctx.synchronize()
            ctx.timing_reset()
            t0 = time.perf_counter()
            for _ in range(steps):
                epoch()
            ctx.synchronize()
            ms = (time.perf_counter() - t0) / steps * 1e3
            tm = {k: ctx.timing(k)[0] / steps for k in NAMES}
            line = {"workload": wl, "N": N, "rank": r, "ms_per_epoch": ms,
                    "shard_user": ctx.shard_range(fh.SIDE_USER),
                    "shard_item": ctx.shard_range(fh.SIDE_ITEM), "kernel_ms": tm}
            print(json.dumps(line), flush=True)
            per_rank.append(ms)
            ctx.close()
        summary[N] = {"max_ms": max(per_rank), "mean_ms": float(np.mean(per_rank))}
    if only:
        return
    if only_n:
        print(json.dumps({"summary": summary}), flush=True)
        return
    t1 = summary[1]["max_ms"]
    for N, s in summary.items():
        s["ideal_ms"] = t1 / N
        s["efficiency_wo_exchange"] = t1 / N / s["max_ms"]
    print(json.dumps({"summary": summary}), flush=True)


if __name__ == "__main__":
    main()
