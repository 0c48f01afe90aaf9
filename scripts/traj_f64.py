#!/usr/bin/env python3
"""Attribution of the l2_reg_exp = 0 trajectory maxima (CPU, diagnostics):
the 3-epoch ML-1M iALS trajectory of tests/test_models_gpu.py::
test_ials_reg_exp0_trajectory_matches_oracle in float64 from the same seeded
initial embeddings, against which both fp32 trajectories -- the oracle's
(oracle/frecsys_oracle.c) and the GPU's (the model_dump file the test copies
when PARITY_DUMP_DIR is set) -- are measured.  If the GPU's distance to the
float64 trajectory is no larger than the oracle's, the GPU-vs-oracle
difference is the fp32 sensitivity of the trajectory itself (two fp32
computations of it differ by that much whatever their order), not an error of
one kernel.

Usage: traj_f64.py <dump.bin> <dim> [out.json]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "safer2-recommender_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402  (test infrastructure: the checker)
from frecsys_hip.data import Dataset  # noqa: E402

REG, W, ALPHA, EPOCHS = 0.003, 0.1, 0.3, 3  # test_models_gpu.py CASES["ials"]


def rel_rows(x, ref):
    num = np.linalg.norm(x.astype(np.float64) - ref, axis=1)
    den = np.linalg.norm(ref, axis=1)
    return np.where(den > 0, num / np.maximum(den, 1e-30), num)


def read_dump(path):
    raw = open(path, "rb").read()
    nu, ni, d = np.frombuffer(raw[:24], np.int64)
    f = np.frombuffer(raw[24:], np.float32)
    return f[:nu * d].reshape(nu, d), f[nu * d:nu * d + ni * d].reshape(ni, d)


def step64(ptr, col, X, out):
    """One iALS side step in float64, lambda = reg (l2_reg_exp = 0,
    ials.h:310-315); rows with an empty history keep their values."""
    G = X.T @ X
    d = X.shape[1]
    M = W * G + REG * np.eye(d)
    for e in range(len(ptr) - 1):
        h = col[ptr[e]:ptr[e + 1]]
        if len(h) == 0:
            continue
        Xh = X[h]
        out[e] = np.linalg.solve(M + Xh.T @ Xh, Xh.sum(0))
    return out


def main():
    dump, dim = sys.argv[1], int(sys.argv[2])
    out = sys.argv[3] if len(sys.argv) > 3 else None
    tr = Dataset.from_csv(os.path.join(ROOT, "tests", "golden", "ml-1m", "train.csv"))
    up, uc = tr.by_user()
    ip, ic = tr.by_item()
    nu, ni = tr.max_user + 1, tr.max_item + 1
    m = O.Model(O.MODEL_IALS, dim, nu, ni, reg=REG, w=W, alpha=ALPHA, reg_exp=0.0, seed=1)
    m.set_data(up, uc, ip, ic)
    m.initialize()
    U0, V0 = m.embeddings()
    U64, V64 = U0.astype(np.float64), V0.astype(np.float64)
    rec = {"dim": dim, "epochs": [], "dump": os.path.basename(dump)}
    for e in range(EPOCHS):
        t = time.time()
        assert m.train() == 0
        U64 = step64(up, uc, V64, U64)
        V64 = step64(ip, ic, U64, V64)
        Uo, Vo = m.embeddings()
        ep = {"epoch": e + 1, "oracle_vs_f64_u": float(rel_rows(Uo, U64).max()),
              "oracle_vs_f64_v": float(rel_rows(Vo, V64).max())}
        rec["epochs"].append(ep)
        print(ep, f"({time.time() - t:.0f} s)", flush=True)
    Ug, Vg = read_dump(dump)
    rec.update(gpu_vs_f64_u=float(rel_rows(Ug, U64).max()),
               gpu_vs_f64_v=float(rel_rows(Vg, V64).max()),
               gpu_vs_oracle_u=float(rel_rows(Ug, Uo.astype(np.float64)).max()),
               gpu_vs_oracle_v=float(rel_rows(Vg, Vo.astype(np.float64)).max()))
    print(json.dumps(rec))
    if out:
        json.dump(rec, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
