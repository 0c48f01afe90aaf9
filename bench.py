#!/usr/bin/env python3
"""bench.py -- iALS closed-form solve loop on MI355X (BASELINE.json configs[1]).

Workload (N=1 and every N): iALS, dim 256, ML-20M-shaped synthetic data
(116,677 users x 20,108 items, ~8.54M interactions, seed 98765; README.md:84
hyperparameters w=0.1, l2_reg=0.003), embeddings N(0, 0.1/sqrt(d)) seed 1.
A "step" is one full Train() epoch (ials.h:187-206 with print_train_stats
off): U half-step (G_V, solve all users, all-gather U), V half-step (G_U,
solve all items, all-gather V), G_V + ComputeUserLoss.  Inputs are resident
in HBM before the timed region.  With N GPUs (torchrun, one process per GPU)
users and items are split nnz-balanced across ranks, Gramian partials are
all-reduced and factor shards all-gathered over RCCL: the total work is
fixed, so scaling is "strong".

value = users updated per second of training wall time = N_users * K / T,
T = max over ranks of the K-epoch wall time.  sec_per_epoch = T / K.

roofline: the dominant kernel is solve_tiled_kernel<8, false, true>, the
d x d solve of the long histories (h > 256; the shorter ones take the
history-space path): gather + MFMA assembly (its fp32
products on the bf16 matrix cores as 3-piece splits, fp32-accurate) +
dataflow blocked Cholesky, compute-bound, priced against the fp32 MFMA
peak (157.3 TFLOP/s) since the algorithm is fp32.
Algorithmic flops per launch = sum over its entities of h*d*(d+1) (0 for
the histories > 2048 rows whose SYRK the split kernel did) + d^3/3 + 2*d^2
(SURVEY 8(d)); duration = its HIP-event time (both half-steps averaged).
`paths` reports the same figures for the other kernels of the epoch.

cpu_baseline: the CPU restatement (oracle/, "port") timing the same U
half-step on a bounded contiguous sample of users, threads = the box's CPU
share (OMP_NUM_THREADS, 16 on the GPU box).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "safer2-recommender_amd"))

import frecsys_hip as fh  # noqa: E402
from frecsys_hip.data import SHAPES, synthetic  # noqa: E402

PEAK_FP32_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix/vector peak (spec)
PEAK_HBM_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--shape", default="ml20m")
    ap.add_argument("--dim", type=int, default=256)
    ap.add_argument("--reg", type=float, default=0.003)
    ap.add_argument("--uobs_weight", type=float, default=0.1)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target CPU-baseline sample duration (0 disables)")
    ap.add_argument("--quiet", action="store_true")
    return ap.parse_args()


def log(msg, rank=0):
    if rank == 0:
        print(msg, file=sys.stderr, flush=True)


def ials_epoch(ctx, args, gv_fresh):
    """One IALSRecommender::Train (ials.h:187-206) over the C-ABI."""
    if not gv_fresh:
        ctx.gramian(fh.SIDE_ITEM, fetch=False)                 # ials.h:321 (V)
    ctx.solve_side(fh.SIDE_USER, fh.KIND_IALS, args.reg, args.uobs_weight)
    ctx.gramian(fh.SIDE_USER, fetch=False)                     # ials.h:321 (U)
    ctx.solve_side(fh.SIDE_ITEM, fh.KIND_IALS, args.reg, args.uobs_weight)
    ctx.gramian(fh.SIDE_ITEM, fetch=False)                     # ials.h:371
    ctx.user_loss(fh.SIDE_USER, args.uobs_weight, False, fetch=False)


def cpu_baseline(up, uc, V, args, nthreads):
    """Oracle U half-step on a bounded contiguous user sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    G = O.gramian(V, nthreads=nthreads)
    n = len(up) - 1
    # calibrate on a small sample, then size the sample to ~cpu_seconds
    k = min(n, 256)
    t0 = time.perf_counter()
    O.step(up[:k + 1], uc[:up[k]], V, G, 0, args.reg, args.uobs_weight, nthreads=nthreads)
    dt = time.perf_counter() - t0
    k2 = int(min(n, max(k, k * args.cpu_seconds / max(dt, 1e-6))))
    t0 = time.perf_counter()
    _, rc = O.step(up[:k2 + 1], uc[:up[k2]], V, G, 0, args.reg, args.uobs_weight,
                   nthreads=nthreads)
    dt = time.perf_counter() - t0
    return {"value": k2 / dt, "unit": "user-solve updates/s", "cores": nthreads, "kind": "port",
            "sample": f"oracle iALS U half-step (Gramian excluded) on users 0..{k2 - 1} of the "
                      f"same synthetic ML-20M-shaped data, d={args.dim}, {dt:.1f} s"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local_rank)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        dist = tdist

    shape = SHAPES[args.shape]
    t0 = time.time()
    up, uc, ip, ic = synthetic(shape)
    nu, ni = len(up) - 1, len(ip) - 1
    nnz = int(up[-1])
    log(f"[bench] data {args.shape}: {nu} users x {ni} items, nnz {nnz} "
        f"({time.time() - t0:.1f}s)", rank)

    ctx = fh.Context(args.dim, nu, ni, device=local_rank)
    if world > 1:
        import torch
        obj = [fh.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        ctx.comm_init(world, rank, obj[0])
    ctx.load_csr(fh.SIDE_USER, up, uc)
    ctx.load_csr(fh.SIDE_ITEM, ip, ic)
    ctx.init_embeddings(1, 0.1)

    def barrier():
        ctx.synchronize()
        if dist is not None:
            dist.barrier()

    ctx.gramian(fh.SIDE_ITEM, fetch=False)
    gv_fresh = True
    for _ in range(args.warmup):
        ials_epoch(ctx, args, gv_fresh)
    ctx.timing_reset()
    barrier()
    t_start = time.perf_counter()
    for s in range(args.steps):
        ials_epoch(ctx, args, gv_fresh)
        if not args.quiet:
            log(f"[bench] step {s + 1}/{args.steps} done", rank)
    barrier()
    elapsed = time.perf_counter() - t_start
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    K = args.steps
    d = args.dim
    Dp = fh.padded_dim(d)
    names = ["solve_user", "solve_item", "gramian", "user_loss", "allgather", "allreduce"]
    names += [f"{s}.{p}" for s in ("solve_user", "solve_item")
              for p in ("dspace", "split", "basis", "hspace", "rotate")]
    timers = {k: ctx.timing(k) for k in names}

    # d-space entities of this rank (iALS: h_eff = h), split ones (> 2 * 1024)
    dual_max = int(os.environ.get("FRECSYS_DUAL_MAX_H", "256"))
    split_rows = int(os.environ.get("FRECSYS_SPLIT_ROWS", "1024"))
    dual_on = os.environ.get("FRECSYS_DUAL", "1") != "0" and Dp >= 64
    chol = d ** 3 / 3.0 + 2.0 * d * d
    fin_flops, fin_ms, fin_n = 0.0, 0.0, 0
    paths = {}
    for side, ptr, name in ((fh.SIDE_USER, up, "solve_user"), (fh.SIDE_ITEM, ip, "solve_item")):
        lo_, hi_ = ctx.shard_range(side)
        hs = np.diff(ptr)[lo_:hi_].astype(np.float64)
        hs = hs[hs > 0]
        ds = hs[hs > dual_max] if dual_on else hs
        unsplit = ds[ds <= 2 * split_rows] if split_rows > 0 else ds
        split = ds[ds > 2 * split_rows] if split_rows > 0 else ds[:0]
        f_fin = float(np.sum(unsplit) * d * (d + 1) + len(ds) * chol)
        ms, n = timers[name + ".dspace"]
        if n:
            fin_flops += f_fin * n / max(K, 1)
            fin_ms += ms
            fin_n += n
        hsp = hs[hs <= dual_max] if dual_on else hs[:0]
        hp = 32.0 * np.ceil(hsp / 32.0)
        paths[name] = {
            "dspace_entities": int(len(ds)), "dspace_ms": ms / max(K, 1),
            "dspace_tflops": f_fin / (ms / max(n, 1) * 1e-3) / 1e12 if n else None,
            "split_rows_total": float(np.sum(split)),
            "split_ms": timers[name + ".split"][0] / max(K, 1),
            "split_tflops": (float(np.sum(split)) * d * (d + 1)
                             / (timers[name + ".split"][0] / max(timers[name + ".split"][1], 1)
                                * 1e-3) / 1e12) if timers[name + ".split"][1] else None,
            "hspace_entities": int(len(hsp)), "hspace_ms": timers[name + ".hspace"][0] / max(K, 1),
            # history-space algorithmic flops: h_p^2 * Dp (SYRK of S) + h_p^3 / 3
            "hspace_tflops": (float(np.sum(hp * hp * Dp + hp ** 3 / 3.0))
                              / (timers[name + ".hspace"][0] / max(K, 1) * 1e-3) / 1e12)
            if timers[name + ".hspace"][1] else None,
            "basis_ms": timers[name + ".basis"][0] / max(K, 1),
            "rotate_ms": timers[name + ".rotate"][0] / max(K, 1),
        }
    avg_ms = fin_ms / max(fin_n, 1)
    flops = fin_flops / max(fin_n / max(K, 1), 1)  # per launch
    achieved_tf = flops / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    n_own = ctx.shard_range(fh.SIDE_USER)[1] - ctx.shard_range(fh.SIDE_USER)[0]
    su_ms = timers["solve_user"][0] / max(K, 1)
    h_all = np.diff(up).astype(np.float64)
    gather_bytes = float(h_all.sum() * d * 4 + h_all.sum() * 4 + (n_own + 1) * 8 + n_own * d * 4)
    gather_gbs = gather_bytes / (su_ms * 1e-3) / 1e9 if su_ms > 0 else 0.0

    traffic = None
    traffic_src = None
    pmc = os.path.join(ROOT, "profiles", "latest_pmc.json")
    if os.path.exists(pmc) and world == 1:
        try:
            js = json.load(open(pmc))
            traffic = js.get("dspace_traffic_bytes")
            traffic_src = js.get("source")
        except Exception:
            traffic = None
    if rank == 0:
        cpu = None
        if args.cpu_seconds > 0 and world == 1:
            nthreads = min(int(os.environ.get("OMP_NUM_THREADS", "16") or 16), os.cpu_count() or 1)
            V = ctx.get_embeddings(fh.SIDE_ITEM)
            try:
                cpu = cpu_baseline(up, uc, V, args, nthreads)
            except Exception as e:  # the baseline must never kill the bench line
                log(f"[bench] cpu baseline failed: {e}")
        line = {
            "metric": "user-solve updates/sec + sec/epoch, iALS dim=256 ML-20M shape",
            "value": nu * K / elapsed,
            "unit": "user-solve updates/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": elapsed / K * 1e3,
            "sec_per_epoch": elapsed / K,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (ML-20M-shaped, Zipf-Mandelbrot items, lognormal users, seed 98765)",
            "config": {"workload": f"iALS d={d} {args.shape}-shaped synthetic, full Train() epoch",
                       "n_users": nu, "n_items": ni, "nnz": nnz, "dim": d, "padded_dim": Dp,
                       "l2_reg": args.reg, "uobs_weight": args.uobs_weight,
                       "parallelism": f"entity-sharded x{world}"},
            "u_halfstep_solve_updates_per_s": (n_own / (su_ms * 1e-3)) * world if su_ms else None,
            "kernel_ms_per_epoch": {k: v[0] / max(K, 1) for k, v in timers.items()},
            "roofline": {"bound": "mfma",
                         "kernel": "solve_tiled_kernel<8, false, true> (d-space solve: split-bf16 "
                                   "MFMA SYRK + fp32 dataflow Cholesky)",
                         "achieved": achieved_tf, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved_tf / PEAK_FP32_TFLOPS, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "avg_launch_ms": avg_ms, "flops_per_launch": flops},
            "paths": paths,
            "gather_roofline": {"bound": "hbm", "scope": "whole user half-step",
                                "achieved": gather_gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                                "frac": gather_gbs / PEAK_HBM_GBS, "bytes_per_step": gather_bytes},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
