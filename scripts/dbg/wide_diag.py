import os, sys
sys.path[:0] = ['oracle', 'safer2-recommender_amd', 'tests']
import numpy as np
import oracle as O
import frecsys_hip as fh
from conftest import make_quirk_data, rel_rows
from test_parity_gpu import _ctx
nu, ni, up, uc, ip, ic = make_quirk_data(n_users=400, n_items=300, hot_frac=(0.40, 0.19, 0.29, 0.186, 0.7))
hu = np.diff(up)
for dim in (500, 512, 1024):
    for mode in ("0", "1"):
        os.environ["FRECSYS_DUAL"] = mode
        ctx, U, V = _ctx(dim, nu, ni, up, uc, ip, ic)
        ctx.gramian(fh.SIDE_ITEM)
        ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, 0.003, 0.1)
        Ug = ctx.get_embeddings(fh.SIDE_USER)
        Uo, rc = O.step(up, uc, V, O.gramian(V), 0, 0.003, 0.1, out=U.copy())
        e = rel_rows(Ug, Uo)
        bad = np.where(e > 1e-4)[0]
        print(dim, "dual" if mode == "1" else "dspace", "max", e.max(), "nbad", len(bad),
              "h of bad", sorted(set(hu[bad].tolist()))[:20], flush=True)
