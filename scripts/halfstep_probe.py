#!/usr/bin/env python3
"""One half-step of a bench workload, bracketed by marker kernels, for
rocprofv3 counter passes (diagnostics; scripts/pmc_halfstep.py reads them).

The context is brought to the state of an epoch's item (or user) half-step:
seeded init, G_V, the user half-step, G_U.  Then a marker kernel
(debug_diag_kernel, via frecsys_debug_diag_factor), `reps` half-steps of the
chosen side, a second marker.  Every dispatch between the markers belongs to
the half-steps.  The library's own event timer of the half-step and its
algorithmic gather bytes (frecsys_work) go to stdout as JSON.

Usage: halfstep_probe.py <workload> <side: user|item> [reps]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "safer2-recommender_amd"))
sys.path.insert(0, ROOT)

import frecsys_hip as fh  # noqa: E402
from frecsys_hip.data import SHAPES, synthetic  # noqa: E402
from bench import WORKLOADS, gather_bytes  # noqa: E402


def main():
    wl, side_name = sys.argv[1], sys.argv[2]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    spec = WORKLOADS[wl]
    assert spec["model"] == "ials", "iALS workloads only"
    f = spec["flags"]
    up, uc, ip, ic = synthetic(SHAPES[spec["shape"]])
    nu, ni = len(up) - 1, len(ip) - 1
    d = spec["dim"]
    ctx = fh.Context(d, nu, ni)
    ctx.load_csr(fh.SIDE_USER, up, uc)
    ctx.load_csr(fh.SIDE_ITEM, ip, ic)
    ctx.init_embeddings(1, 0.1)
    solve = lambda s: ctx.solve_side(s, fh.KIND_IALS, f["l2_reg"], f["uobs_weight"],  # noqa: E731
                                     reg_exp=f["l2_reg_exp"])
    ctx.gramian(fh.SIDE_ITEM, fetch=False)
    solve(fh.SIDE_USER)
    ctx.gramian(fh.SIDE_USER, fetch=False)
    side = fh.SIDE_ITEM if side_name == "item" else fh.SIDE_USER
    if side == fh.SIDE_USER:
        solve(fh.SIDE_ITEM)
        ctx.gramian(fh.SIDE_ITEM, fetch=False)
    marker = np.eye(32, dtype=np.float32)[None]
    ctx.synchronize()
    ctx.timing_reset()
    ctx.debug_diag_factor(marker, True)  # marker kernel: debug_diag_kernel
    for _ in range(reps):
        solve(side)
    ctx.synchronize()
    ctx.debug_diag_factor(marker, True)
    name = "solve_item" if side == fh.SIDE_ITEM else "solve_user"
    ms, n = ctx.timing(name)
    ptr = ip if side == fh.SIDE_ITEM else up
    other_rows = nu if side == fh.SIDE_ITEM else ni
    out = {"workload": wl, "side": side_name, "reps": reps, "halfstep_ms": ms / max(n, 1),
           "algorithmic_gather_bytes": gather_bytes(ptr, 0, len(ptr) - 1, d, d),
           "gathered_table_bytes": other_rows * fh.padded_dim(d) * 4,
           "dspace_ms": ctx.timing(name + ".dspace")[0] / reps,
           "hspace_ms": ctx.timing(name + ".hspace")[0] / reps}
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
