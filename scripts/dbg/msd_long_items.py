"""Diagnostic: GPU vs oracle vs float64 truth on the longest MSD items (d=512, iALS V step)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ("safer2-recommender_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np
import frecsys_hip as fh
import oracle as O
from frecsys_hip.data import SHAPES, synthetic

up, uc, ip, ic = synthetic(SHAPES["msd"])
nu, ni = len(up) - 1, len(ip) - 1
d, reg, w = 512, 0.002, 0.05
ctx = fh.Context(d, nu, ni)
ctx.load_csr(fh.SIDE_USER, up, uc); ctx.load_csr(fh.SIDE_ITEM, ip, ic)
ctx.init_embeddings(1, 0.1)
ctx.gramian(fh.SIDE_ITEM, fetch=False)
ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, reg, w)
Ug = ctx.get_embeddings(fh.SIDE_USER)
Gg = ctx.gramian(fh.SIDE_USER)
ctx.solve_side(fh.SIDE_ITEM, fh.KIND_IALS, reg, w)
Vg = ctx.get_embeddings(fh.SIDE_ITEM)
h = np.diff(ip)
rows = np.sort(np.argsort(-h)[:4])
rows = np.concatenate([rows, np.nonzero((h > 2000) & (h < 3000))[0][:2]])
rp = np.concatenate([[0], np.cumsum(h[rows])]).astype(np.int64)
cl = np.concatenate([ic[ip[r]:ip[r + 1]] for r in rows]).astype(np.int32)
Go = O.gramian(Ug)
Vo, rc = O.step(rp, cl, Ug, Go, 0, reg, w)
U64 = Ug.astype(np.float64)
G64 = U64.T @ U64
print("G gpu vs fp64 rel %.2e, oracle G vs fp64 %.2e" % (np.abs(Gg - G64).max() / np.abs(G64).max(), np.abs(Go - G64).max() / np.abs(G64).max()))
for k, r in enumerate(rows):
    X = U64[ic[ip[r]:ip[r + 1]]]
    hh = len(X)
    lam = reg * (hh + w * nu)
    A = w * G64 + lam * np.eye(d) + X.T @ X
    b = X.sum(0)
    x = np.linalg.solve(A, b)
    n = np.linalg.norm(x)
    bf = X.astype(np.float32).sum(0, dtype=np.float32)  # numpy pairwise fp32
    print("item %d h %d: gpu-fp64 %.2e oracle-fp64 %.2e gpu-oracle %.2e cond %.3e |b| %.3f |x| %.4f"
          % (r, hh, np.linalg.norm(Vg[r] - x) / n, np.linalg.norm(Vo[k] - x) / n,
             np.linalg.norm(Vg[r] - Vo[k]) / np.linalg.norm(Vo[k]), np.linalg.cond(A), np.linalg.norm(b), n), flush=True)
