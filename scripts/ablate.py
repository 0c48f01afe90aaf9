"""Diagnostic: time the solve kernel with phases skipped (FRECSYS_DEBUG_SKIP).
Results of skipped runs are garbage; only the timings matter."""
import os, sys, json, time, subprocess
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "safer2-recommender_amd"))
if len(sys.argv) > 1 and sys.argv[1] == "child":
    import numpy as np
    import frecsys_hip as fh
    from frecsys_hip.data import SHAPES, synthetic
    d = int(os.environ.get("DIM", "256"))
    up, uc, ip, ic = synthetic(SHAPES[os.environ.get("SHAPE", "ml20m")])
    ctx = fh.Context(d, len(up) - 1, len(ip) - 1)
    ctx.load_csr(0, up, uc); ctx.load_csr(1, ip, ic); ctx.init_embeddings(1, 0.1)
    ctx.gramian(1, fetch=False); ctx.gramian(0, fetch=False)
    for side in (0, 1):
        try:
            ctx.solve_side(side, 0, 0.003, 0.1)
        except fh.FrecsysError:
            pass
    ctx.timing_reset()
    for _ in range(2):
        for side in (0, 1):
            try:
                ctx.solve_side(side, 0, 0.003, 0.1)
            except fh.FrecsysError:
                pass
    out = {"mask": int(os.environ.get("FRECSYS_DEBUG_SKIP", "0"))}
    for side in ("solve_user", "solve_item"):
        for part in ("", ".dspace", ".basis", ".hspace", ".rotate"):
            out[side + part] = round(ctx.timing(side + part)[0] / 2, 3)
    print(json.dumps(out))
    sys.exit(0)
for mask in [int(m) for m in (sys.argv[1:] or ["0", "1", "2", "4", "8", "16", "30", "31"])]:
    env = dict(os.environ, FRECSYS_DEBUG_SKIP=str(mask), FRECSYS_DUAL_SERIAL="1")
    out = subprocess.run([sys.executable, __file__, "child"], env=env, capture_output=True, text=True, timeout=300)
    print(out.stdout.strip() or out.stderr[-500:], flush=True)
