"""Two iALS epochs at several dims on the test suite's quirk data with the
library in the tree; writes every U, V to an .npz (for a bitwise A/B of two
library builds run one after the other)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "safer2-recommender_amd"), ROOT]
from conftest import make_quirk_data  # noqa: E402
import frecsys_hip as fh  # noqa: E402
import oracle as O  # noqa: E402

nu, ni, up, uc, ip, ic = make_quirk_data()
res = {}
for dim in (64, 128, 256, 512):
    ctx = fh.Context(dim, nu, ni, parity_quirks=True)
    ctx.load_csr(fh.SIDE_USER, up, uc)
    ctx.load_csr(fh.SIDE_ITEM, ip, ic)
    U, V = O.init_embeddings(1, 0.1, dim, nu, ni)
    ctx.set_embeddings(fh.SIDE_USER, U)
    ctx.set_embeddings(fh.SIDE_ITEM, V)
    for _ in range(2):
        ctx.gramian(fh.SIDE_ITEM)
        ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, 0.003, 0.1)
        ctx.gramian(fh.SIDE_USER)
        ctx.solve_side(fh.SIDE_ITEM, fh.KIND_IALS, 0.003, 0.1)
    res[f"U{dim}"] = ctx.get_embeddings(fh.SIDE_USER)
    res[f"V{dim}"] = ctx.get_embeddings(fh.SIDE_ITEM)
    ctx.close()
np.savez(sys.argv[1], **res)
print("saved", sys.argv[1])
