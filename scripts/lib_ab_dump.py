"""Dump (every 97th word of) the d-space solve outputs of one libfrecsys_hip.so build, for a
bit-for-bit A/B of two builds of the same kernels (e.g. -DFRECSYS_SYRK_SB=0
against the default):  python3 scripts/lib_ab_dump.py <lib.so> <out.npz>
Every entity on the d-space path (FRECSYS_DUAL=0), long histories through
the split slabs (FRECSYS_SPLIT_ROWS=64), the solve kinds and both sides at
d = 256 and 128 on a 20K x 5K Zipf-shaped set."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "safer2-recommender_amd"))
import frecsys_hip as fh  # noqa: E402
from frecsys_hip.data import SynthShape, synthetic  # noqa: E402

os.environ.setdefault("FRECSYS_DUAL", "0")  # FRECSYS_DUAL=1: the history-space path too
os.environ["FRECSYS_SPLIT_ROWS"] = "64"
fh.load_library(sys.argv[1])
shape = SynthShape(20_000, 5_000, 1_000_000, min_uc=5)
up, uc, ip, ic = synthetic(shape, seed=5)[:4]
out = {}
for dim in (256, 128):
    ctx = fh.Context(dim, shape.n_users, shape.n_items, device=0)
    ctx.load_csr(fh.SIDE_USER, up, uc)
    ctx.load_csr(fh.SIDE_ITEM, ip, ic)
    ctx.init_embeddings(1, 0.1)
    om = (0.05 + 0.95 * np.random.default_rng(5).random(shape.n_users)).astype(np.float32)
    h = np.diff(up).astype(np.float32)
    nu_w = np.where(h > 0, om / np.maximum(h, 1), 0).astype(np.float32)
    item_reg = (0.5 + np.random.default_rng(6).random(shape.n_items)).astype(np.float32)
    ctx.gramian(fh.SIDE_ITEM, fetch=False)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, 0.003, 0.1)
    out[f"u_ials_{dim}"] = ctx.get_embeddings(fh.SIDE_USER)
    ctx.gramian(fh.SIDE_USER, fetch=False)
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_IALS, 0.003, 0.1)
    out[f"v_ials_{dim}"] = ctx.get_embeddings(fh.SIDE_ITEM)
    ctx.gramian(fh.SIDE_ITEM, fetch=False)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_WEIGHTED_U, 0.003, 0.1, entity_weight=om)
    out[f"u_w_{dim}"] = ctx.get_embeddings(fh.SIDE_USER)
    ctx.gramian(fh.SIDE_USER, weights=om, fetch=False)
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_WEIGHTED_V, 0.003, 0.1, alpha=0.3, entity_reg=item_reg,
                   other_weight=nu_w)
    out[f"v_w_{dim}"] = ctx.get_embeddings(fh.SIDE_ITEM)
    ctx.close()
np.savez_compressed(sys.argv[2], **{k: np.frombuffer(v.tobytes(), np.uint32)[::97] for k, v in out.items()})
print("dumped", sys.argv[2], {k: float(np.abs(v).max()) for k, v in out.items()})
