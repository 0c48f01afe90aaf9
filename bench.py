#!/usr/bin/env python3
"""bench.py -- the closed-form solve loop on MI355X, timed through the product's
own Train() (include/frecsys_model.h -> the C++ model classes -> libfrecsys_hip.so).

Headline (the JSON line's top level; BASELINE.json configs[1]): iALS, dim 256,
ML-20M-shaped synthetic data (116,677 users x 20,108 items, ~8.54M interactions,
seed 98765), README.md:84 hyperparameters (w=0.1, l2_reg=0.003, reg_exp 1),
stdev 0.1, init seed 1, print_train_stats 0.  A "step" is one
`IALSRecommender::Train()` call (ials.h:187-206): U half-step (Gramian of V,
solve all users, all-gather U), V half-step, Gramian + ComputeUserLoss.  Inputs
are resident in HBM before the timed region.  With N GPUs (torchrun, one process
per GPU) users and items are split nnz-balanced across ranks, Gramian partials
all-reduced and factor shards all-gathered over RCCL: the total work is fixed
("strong" scaling).

value = users updated per second of training wall time = N_users * K / T,
T = max over ranks of the K-epoch wall time.  sec_per_epoch = T / K.

`workloads` carries the same measurement for BASELINE configs[2] (SAFER2 d=256
ML-20M-shaped, README.md:79 flags, pd=1 xi=5 use_snr=1 sampling_ratio=0.1) and
configs[3] (iALS d=512 MSD-shaped, README.md:105), each with its own roofline,
gather roofline and cpu_baseline, and configs[4] (SAFER2 d=1024 2M x 500K,
README.md:100; 2 timed epochs) -- all three at every N; `--workload` runs
one of them as the headline.

roofline: the dominant kernel of the workload, priced against the fp32 MFMA peak
(157.3 TFLOP/s; the algorithm is fp32 and compute-bound): algorithmic flops per
launch (h*d*(d+1) SYRK + d^3/3 + 2d^2 solve per d-space entity) /
its HIP-event launch time.  gather_roofline: SURVEY 8(d)'s gather bytes of both
half-steps (nnz*d*4 + nnz*4 + (N+1)*8 + N*d*4 per side) / the solve time of both
half-steps, vs 8 TB/s -- the north-star figure at d=512 on the MSD shape.
loss_gather_roofline: the same bytes of the ComputeUserLoss pass (a pure
embedding gather) / its time.

cpu_baseline: a blocked, vectorised CPU restatement of the reference's Eigen
path (oracle/cpu_baseline.c, kind "port") timing samples of both half-steps
on this host's CPU share, projected to one epoch: users per epoch-second,
like the GPU value.

The shipped library has no knobs that skip work; bench.py refuses to run with
any FRECSYS_* variable set (they select paths for profiling) unless
--allow-env is given, and then records them in the line as "frecsys_env".
"""
import argparse
import json
import os
import platform
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "safer2-recommender_amd"))

# frecsys_hip is imported in main(), after the launcher decision: a parent
# that spawns the N ranks must not have touched the GPU library.
fh = None
SHAPES = synthetic = None

PEAK_FP32_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix peak (spec)
# the products run as 6 bf16 MFMAs per fp32-accurate product (common.h
# mfma_x6): their own ceiling is the dense bf16 peak / 6, in fp32 flops
PEAK_BF16_TFLOPS = 2500.0
PEAK_SPLIT_BF16_TFLOPS = PEAK_BF16_TFLOPS / 6.0
PEAK_HBM_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)

# BASELINE.json configs; flags are the run_model flags (README.md lines cited).
WORKLOADS = {
    "ials_ml20m_d256": dict(
        config=1, model="ials", shape="ml20m", dim=256, readme="README.md:84",
        flags=dict(l2_reg=0.003, uobs_weight=0.1, l2_reg_exp=1.0)),
    "safer2_ml20m_d256": dict(
        config=2, model="safer2", shape="ml20m", dim=256, readme="README.md:79",
        flags=dict(l2_reg=0.002, uobs_weight=0.002, alpha=0.3, bandwidth=0.18, pd_iterations=1,
                   xi_iterations=5, use_snr=True, sampling_ratio=0.1)),
    "ials_msd_d512": dict(
        config=3, model="ials", shape="msd", dim=512, readme="README.md:105",
        flags=dict(l2_reg=0.002, uobs_weight=0.05, l2_reg_exp=1.0)),
    "safer2_2m500k_d1024": dict(
        config=4, model="safer2", shape="2m500k", dim=1024, readme="README.md:100",
        flags=dict(l2_reg=0.0012, uobs_weight=0.0004, alpha=0.3, bandwidth=0.1,
                   pd_iterations=1, xi_iterations=5, use_snr=True, sampling_ratio=0.1),
        max_extra_steps=2),  # ~1.6 s epochs after ~40 s of data generation
}
HEADLINE = "ials_ml20m_d256"
# the other BASELINE configs, at every N: configs[3] and configs[4] are defined
# on 8 GPUs (BASELINE.json), so the driver's N = 1, 2, 4, 8 sweep measures
# them all; config 5 last (its data takes ~40 s per rank)
DEFAULT_EXTRAS = ("safer2_ml20m_d256", "ials_msd_d512", "safer2_2m500k_d1024")


def default_extras(world):
    """The extra workloads of a default run at any world size: BASELINE
    configs 3, 4 and 5 (the CPU baseline is timed at N = 1 only)."""
    del world
    return ",".join(DEFAULT_EXTRAS)


def launch_plan(args, world):
    """What a run of these arguments measures: the rank launch (None when this
    process is already a rank), the headline and the extra workloads."""
    extras = args.extras if args.extras is not None else default_extras(world)
    return {"launch": launch_command(args) if world_from_env(args) is None else None,
            "n_gpus": world, "workload": args.workload,
            "extras": [x for x in extras.split(",") if x and x != args.workload],
            "cpu_baseline": world == 1 and args.cpu_seconds > 0}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default=HEADLINE, choices=sorted(WORKLOADS))
    ap.add_argument("--extras", default=None,
                    help="comma-separated extra workloads measured after the headline "
                         "('' for none; default: the other BASELINE configs 3, 4, 5)")
    ap.add_argument("--extra-steps", type=int, default=3)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target CPU-baseline sample duration per workload (0 disables)")
    ap.add_argument("--allow-env", action="store_true",
                    help="run although FRECSYS_* variables are set (recorded in the line)")
    ap.add_argument("--quiet", action="store_true")
    ap.add_argument("--print-launch", action="store_true",
                    help="print the launch plan (the N-rank command bench.py would run, the "
                         "headline and extra workloads) as JSON and exit")
    return ap.parse_args()


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_command(args):
    """One process per GPU: torch.distributed.run on this node, rendezvous on
    127.0.0.1, the same bench.py arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
            f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]


def world_from_env(args):
    """(world, rank, local_rank) of this process, or None when bench.py must
    launch the ranks itself (--gpus N > 1 without a torchrun environment).
    Exits non-zero when the environment's world size is not --gpus."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus > 1:
            return None
        env_world = "1"
    world = int(env_world)
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a "
                 f"{world}-rank run as {args.gpus} GPUs")
    return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def log(msg, rank=0):
    if rank == 0:
        print(msg, file=sys.stderr, flush=True)


def frecsys_env():
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith("FRECSYS_")}


def host_cpu_share():
    """Threads for the CPU baseline: this process's CPU share (affinity,
    bounded by a cgroup quota and OMP_NUM_THREADS when set), and what the
    host reports."""
    info = {"os_cpu_count": os.cpu_count()}
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    info["affinity"] = aff
    share = aff
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            info["cgroup_quota_cpus"] = float(q) / float(p)
            share = min(share, max(1, int(float(q) / float(p))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        info["omp_num_threads"] = int(omp)
        share = min(share, int(omp))
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                info["model"] = line.split(":", 1)[1].strip()
            if line.startswith("Flags:"):
                info["avx512f"] = " avx512f " in line + " "
    except (OSError, subprocess.SubprocessError):
        info["model"] = platform.processor()
    return share, info


def path_accounting(ctx, timers, K):
    """Algorithmic work per solve path of both half-steps, as the library
    itself accounted it while launching (frecsys_work: SURVEY 8(d) flops and
    bytes per entity of the paths it chose), over the HIP-event times."""
    fin_flops, fin_ms, fin_n = 0.0, 0.0, 0
    paths = {}
    per = lambda x: x / max(K, 1)  # noqa: E731
    for name in ("solve_user", "solve_item"):
        f, b, ne, n = ctx.work(name + ".dspace")
        ms, nt = timers[name + ".dspace"]
        if nt:
            fin_flops += f
            fin_ms += ms
            fin_n += nt
        fs, _, nsplit, _ = ctx.work(name + ".split")
        sp_ms, sp_n = timers[name + ".split"]
        fh_, _, nh, _ = ctx.work(name + ".hspace")
        hs_ms, hs_n = timers[name + ".hspace"]
        paths[name] = {
            "dspace_entities": per(ne), "dspace_ms": per(ms), "dspace_launches_per_step": per(nt),
            "dspace_tflops": f / (ms * 1e-3) / 1e12 if nt and ms > 0 else None,
            "split_entities": per(nsplit), "split_ms": per(sp_ms),
            "split_tflops": fs / (sp_ms * 1e-3) / 1e12 if sp_n and sp_ms > 0 else None,
            "hspace_entities": per(nh), "hspace_ms": per(hs_ms),
            "hspace_tflops": fh_ / (hs_ms * 1e-3) / 1e12 if hs_n and hs_ms > 0 else None,
            "basis_ms": per(timers[name + ".basis"][0]),
            "rotate_ms": per(timers[name + ".rotate"][0]),
        }
    avg_ms = fin_ms / max(fin_n, 1)
    flops = fin_flops / max(fin_n, 1)  # per launch (mean over launches)
    return paths, avg_ms, flops


def gather_bytes(ptr, lo, hi, d, out_floats):
    """SURVEY 8(d) gather bytes of one pass over rows [lo, hi): every history
    row of the other side (d floats) + its int32 id + row_ptr + the output."""
    nnz = float(ptr[hi] - ptr[lo])
    n = hi - lo
    return nnz * d * 4 + nnz * 4 + (n + 1) * 8 + n * out_floats * 4


def load_pmc(workload):
    """The workload's counter summary in profiles/latest_pmc.json (rocprofv3
    FETCH_SIZE / WRITE_SIZE passes, scripts/profile_round.sh), or {}."""
    path = os.path.join(ROOT, "profiles", "latest_pmc.json")
    if not os.path.exists(path):
        return {}, None
    try:
        js = json.load(open(path))
    except (OSError, ValueError):
        return {}, None
    return js.get("workloads", {}).get(workload, {}), js.get("source")


def loss_roofline(pmc, alg_bytes, ms, alg_gbs, table_bytes):
    """ComputeUserLoss, a pure gather of item rows.  `achieved` is the FABRIC
    rate: FETCH_SIZE x 2 + WRITE_SIZE bytes of its gather kernel per pass
    (counters of the tracked profile, L2 misses incl. Infinity-Cache hits)
    over this run's pass time.  The algorithmic rate (SURVEY 8(d) bytes over
    time) is kept beside it; it exceeds the HBM peak whenever the item table
    is served from the caches, so it is never called HBM."""
    fab = pmc.get("loss_fabric_bytes_per_pass")
    out = {"bound": "hbm", "kind": "fabric (L2-miss incl. Infinity Cache)",
           "scope": "ComputeUserLoss gather kernel (loss_gather*)",
           "achieved": None, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": None,
           "traffic": fab, "algorithmic_gbs": alg_gbs, "algorithmic_frac": alg_gbs / PEAK_HBM_GBS,
           "algorithmic_bytes_per_launch": alg_bytes, "gathered_table_bytes": table_bytes}
    if fab and ms > 0:
        out["achieved"] = fab / (ms * 1e-3) / 1e9
        out["frac"] = out["achieved"] / PEAK_HBM_GBS
    return out


def item_gather_fabric(pmc, ms, n_items, Dp):
    """The north-star figure on a table larger than the 256 MiB Infinity
    Cache (MSD: the item half-step gathers the 0.97 GB user table): fabric
    bytes of every kernel of one item half-step (scripts/gather_prof.sh:
    marker-bracketed rocprofv3 FETCH_SIZE x2 + WRITE_SIZE passes) over this
    run's item half-step time, against 8 TB/s."""
    h = pmc.get("halfstep_item")
    if not h or ms <= 0:
        return None
    fab = h["fabric_bytes"]
    return {"bound": "hbm", "kind": "fabric (L2-miss incl. Infinity Cache)",
            "scope": "item half-step, every kernel (gather + workspace traffic)",
            "gathered_table_bytes": h["gathered_table_bytes"],
            "achieved": fab / (ms * 1e-3) / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": fab / (ms * 1e-3) / 1e9 / PEAK_HBM_GBS, "traffic": fab,
            "algorithmic_gather_bytes": h["algorithmic_gather_bytes"],
            "algorithmic_gbs": h["algorithmic_gather_bytes"] / (ms * 1e-3) / 1e9,
            "halfstep_ms": ms}


def cpu_baseline(spec, up, uc, ip, ic, U, V, seconds, nthreads, host):
    """The CPU baseline of one Train() epoch, like for like with the GPU
    `value` (users updated per second of epoch): oracle/cpu_baseline.c (a
    cache-blocked, AVX-512-vectorised restatement of the reference's Eigen
    path: blocked SYRK of 128-row batches, blocked LLT) times a contiguous
    sample of each half-step (U and V, the workload's kinds, Gramians by
    the oracle); each half-step is projected to the whole side by the
    SURVEY 8(d) per-entity cost h d (d+1) + d^3 / 3, and the epoch is the
    sum.  About `seconds` of CPU work in all."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    f = spec["flags"]
    d = spec["dim"]
    nu, ni = len(up) - 1, len(ip) - 1
    hu, hi = np.diff(up).astype(np.float64), np.diff(ip).astype(np.float64)
    t0 = time.perf_counter()
    G_V = O.gramian(V, nthreads=nthreads)
    t_gv = time.perf_counter() - t0
    if spec["model"] == "ials":
        ukw = dict(kind=0, reg=f["l2_reg"], w=f["uobs_weight"], reg_exp=f["l2_reg_exp"])
        vkw = dict(ukw)
        om = None
        t0 = time.perf_counter()
        G_U = O.gramian(U, nthreads=nthreads)
        t_gu = time.perf_counter() - t0
    else:  # ProjectU with omega = alpha, ProjectV with nu = omega / |H_u| (the first epoch)
        om = np.full(nu, f["alpha"], np.float32)
        hs = np.where(hu > 0, hu, 1.0)
        nu_w = (om / hs).astype(np.float32)
        item_reg = np.add.reduceat((1.0 / hs)[ic], ip[:-1]).astype(np.float32)
        item_reg[hi == 0] = 0.0
        ukw = dict(kind=1, reg=f["l2_reg"], w=f["uobs_weight"], entity_weight=om)
        vkw = dict(kind=2, reg=f["l2_reg"], w=f["uobs_weight"], alpha=f["alpha"],
                   entity_reg=item_reg, other_weight=nu_w)
        t0 = time.perf_counter()
        G_U = O.gramian(U, om, nthreads=nthreads)
        t_gu = time.perf_counter() - t0

    def cost(h):
        return float(np.sum(np.where(h > 0, h * d * (d + 1.0) + d ** 3 / 3.0, 0.0)))

    def half(ptr, col, X, G, kw, n, budget):
        def run(k):
            ex = {kk: (vv[:k] if kk in ("entity_weight", "entity_reg") else vv)
                  for kk, vv in kw.items()}
            t = time.perf_counter()
            O.baseline_step(ptr[:k + 1], col[:ptr[k]], X, G, nthreads=nthreads, **ex)
            return time.perf_counter() - t
        k = min(n, 64)
        dt = run(k)
        k2 = int(min(n, max(k, k * budget / max(dt, 1e-6))))
        dt = run(k2)
        h = np.diff(ptr)
        return k2, dt, dt * cost(h) / max(cost(h[:k2]), 1.0)

    ku, dtu, tu = half(up, uc, V, G_V, ukw, nu, seconds / 2)
    kv, dtv, tv = half(ip, ic, U, G_U, vkw, ni, seconds / 2)
    epoch = tu + tv + t_gu + t_gv
    return {"value": nu / epoch, "unit": "user-solve updates/s", "cores": nthreads,
            "kind": "port", "host": host,
            "sec_per_epoch_projected": epoch,
            "u_halfstep_updates_per_s": ku / dtu,
            "sample": f"oracle/cpu_baseline.c (blocked, AVX-512-vectorised restatement of the "
                      f"reference's Eigen path) on {nthreads} threads: U half-step on users "
                      f"0..{ku - 1} ({dtu:.1f} s) and V half-step on items 0..{kv - 1} "
                      f"({dtv:.1f} s) of the same synthetic {spec['shape']}-shaped data, "
                      f"d={d}, each projected to its whole side by sum(h d (d+1) + d^3/3), "
                      f"plus both Gramians timed whole ({t_gu + t_gv:.1f} s); epoch "
                      f"{epoch:.2f} s projected; not Eigen itself"}


def run_workload(name, args, world, rank, local_rank, dist, data_cache, steps, warmup, cpu_s):
    spec = WORKLOADS[name]
    t0 = time.time()
    if spec["shape"] not in data_cache:
        data_cache.clear()  # one shape resident at a time
        data_cache[spec["shape"]] = synthetic(SHAPES[spec["shape"]])
    up, uc, ip, ic = data_cache[spec["shape"]]
    nu, ni = len(up) - 1, len(ip) - 1
    nnz = int(up[-1])
    log(f"[bench] {name}: data {nu} users x {ni} items, nnz {nnz} ({time.time() - t0:.1f}s)", rank)
    users = np.repeat(np.arange(nu, dtype=np.int32), np.diff(up))
    cid = None
    if world > 1:
        obj = [fh.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        cid = obj[0]
    model = fh.Model(spec["model"], users, uc, dim=spec["dim"], stdev=0.1, seed=1,
                     print_train_stats=False, device=local_rank, world=world, rank=rank,
                     comm_id=cid, **spec["flags"])
    del users
    ctx = model.context()
    cw, _, comm_ranks = ctx.comm_world()
    if world > 1 and (cw != world or comm_ranks != world):
        raise SystemExit(f"bench.py: the model joined world {cw} with an RCCL communicator of "
                         f"{comm_ranks} ranks, expected {world}")
    model.initialize()  # run_model.cc:246-257 (SAFER2); outside the timed region

    def barrier():
        ctx.synchronize()
        if dist is not None:
            dist.barrier()

    model.train(warmup)
    ctx.timing_reset()
    barrier()
    t_start = time.perf_counter()
    for s in range(steps):
        model.train(1)
        if not args.quiet:
            log(f"[bench] {name} step {s + 1}/{steps} done", rank)
    barrier()
    elapsed = time.perf_counter() - t_start
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    K = steps
    d = spec["dim"]
    Dp = fh.padded_dim(d)
    names = ["solve_user", "solve_item", "gramian", "user_loss", "user_loss.gather", "allgather",
             "gram_exchange"]
    names += [f"{s}.{p}" for s in ("solve_user", "solve_item")
              for p in ("dspace", "split", "basis", "hspace", "rotate")]
    timers = {k: ctx.timing(k) for k in names}
    paths, avg_ms, flops = path_accounting(ctx, timers, K)
    achieved_tf = flops / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    ulo, uhi = ctx.shard_range(fh.SIDE_USER)
    ilo, ihi = ctx.shard_range(fh.SIDE_ITEM)
    su_ms = timers["solve_user"][0] / max(K, 1)
    si_ms = timers["solve_item"][0] / max(K, 1)
    gb = gather_bytes(up, ulo, uhi, d, d) + gather_bytes(ip, ilo, ihi, d, d)
    g_gbs = gb / ((su_ms + si_ms) * 1e-3) / 1e9 if su_ms + si_ms > 0 else 0.0
    # the gather kernel's own time (library event pair around it), the
    # kernel the loss_gather roofline prices; the pass (u^T G u + gather)
    # when the library has no separate timer (Dp <= 16)
    lg = timers["user_loss.gather"] if timers["user_loss.gather"][1] else timers["user_loss"]
    loss_ms = lg[0] / max(lg[1], 1)
    lw = ctx.work("user_loss")
    lb = lw[1] / max(lw[3], 1)  # algorithmic bytes per ComputeUserLoss pass (library-accounted)
    l_gbs = lb / (loss_ms * 1e-3) / 1e9 if loss_ms > 0 else 0.0
    pmc, traffic_src = load_pmc(name) if world == 1 else ({}, None)
    traffic = pmc.get("dominant_traffic_bytes")
    wide = Dp > 256
    res = {
        "workload": name,
        "baseline_config": f"BASELINE.json configs[{spec['config']}]",
        "model": spec["model"], "flags": spec["flags"], "flags_source": spec["readme"],
        "n_users": nu, "n_items": ni, "nnz": nnz, "dim": d, "padded_dim": Dp,
        "rccl_ranks": comm_ranks,
        "value": nu * K / elapsed, "unit": "user-solve updates/s",
        "steps": K, "warmup": warmup,
        "ms_per_step": elapsed / K * 1e3, "sec_per_epoch": elapsed / K,
        "u_halfstep_solve_updates_per_s": ((uhi - ulo) / (su_ms * 1e-3)) * world if su_ms else None,
        "kernel_ms_per_epoch": {k: v[0] / max(K, 1) for k, v in timers.items()},
        "roofline": {"bound": "mfma",
                     "kernel": ("wide_syrk3_kernel<2> (slabs of the long histories) + "
                                "wide_syrk3_kernel<1> (split-bf16 MFMA SYRK from the pre-split "
                                "table) + " + ("wide_chol2_kernel<32> (two-panel" if Dp == 1024
                                               else "wide_chol_kernel<16> (") +
                                " batched d-space Cholesky, A in an HBM workspace)") if wide else
                               ("solve_tiled_kernel<8, false, true> (d-space solve: split-bf16 "
                                "MFMA SYRK + fp32 dataflow Cholesky)"),
                     "achieved": achieved_tf, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved_tf / PEAK_FP32_TFLOPS, "traffic": traffic,
                     # the same work against the split-bf16 ceiling the kernels run at
                     "peak_split_bf16": PEAK_SPLIT_BF16_TFLOPS,
                     "frac_split_bf16": achieved_tf / PEAK_SPLIT_BF16_TFLOPS,
                     "traffic_source": traffic_src,
                     "avg_launch_ms": avg_ms, "flops_per_launch": flops},
        "paths": paths,
        # ALGORITHMIC bytes over time: the solve phase is compute-bound (DESIGN
        # 3.7), so this is a work rate, not a measure of HBM traffic
        "gather_roofline": {"bound": "hbm", "kind": "algorithmic",
                            "scope": "both half-steps' solves (SURVEY 8(d) gather bytes / solve "
                                     "time)",
                            "achieved": g_gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                            "frac": g_gbs / PEAK_HBM_GBS, "bytes_per_step": gb},
        "loss_gather_roofline": loss_roofline(pmc, lb, loss_ms, l_gbs, ni * Dp * 4),
    }
    item = item_gather_fabric(pmc, si_ms, ni, Dp)
    if item:
        res["item_gather_fabric"] = item
    # the silent slow path (a side rerun in d-space after a history-space
    # pivot failure or a tagged-poll timeout), over the whole run incl. warmup
    res["hspace_reruns"] = ctx.counter("hspace_reruns")
    res["tagged_timeouts"] = ctx.counter("tagged_timeouts")
    if spec["model"] != "ials":
        res["mean_dual_weight"] = model.mean_weight()
    if cpu_s > 0 and world == 1 and rank == 0:
        try:
            nthreads, host = host_cpu_share()
            U = ctx.get_embeddings(fh.SIDE_USER)
            V = ctx.get_embeddings(fh.SIDE_ITEM)
            res["cpu_baseline"] = cpu_baseline(spec, up, uc, ip, ic, U, V, cpu_s, nthreads, host)
        except Exception as e:  # the baseline must never kill the bench line
            log(f"[bench] cpu baseline failed: {e}")
            res["cpu_baseline"] = None
    else:
        res["cpu_baseline"] = None
    ctx.close()
    model.close()
    return res


def main():
    global fh, SHAPES, synthetic
    args = parse()
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    env = frecsys_env()
    if env and not args.allow_env:
        sys.exit(f"bench.py: refusing to run with {sorted(env)} set (profiling path selectors; "
                 f"pass --allow-env to run anyway, recorded in the line)")
    ranks = world_from_env(args)
    if args.print_launch:
        print(json.dumps(launch_plan(args, args.gpus)))
        return
    if ranks is None:  # launch the N ranks (children) and exit with their status
        sys.exit(subprocess.run(launch_command(args)).returncode)
    world, rank, local_rank = ranks
    import frecsys_hip as fh_mod
    from frecsys_hip import data as fh_data
    fh, SHAPES, synthetic = fh_mod, fh_data.SHAPES, fh_data.synthetic
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local_rank)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        dist = tdist

    data_cache = {}
    head = run_workload(args.workload, args, world, rank, local_rank, dist, data_cache,
                        args.steps, args.warmup, args.cpu_seconds)
    extras = []
    if args.extras is None:
        args.extras = default_extras(world)
    for name in [x for x in args.extras.split(",") if x and x != args.workload]:
        steps = min(args.extra_steps, WORKLOADS[name].get("max_extra_steps", args.extra_steps))
        try:
            extras.append(run_workload(name, args, world, rank, local_rank, dist, data_cache,
                                       steps, 1, args.cpu_seconds))
        except Exception as e:  # an extra never takes the headline line down with it
            log(f"[bench] {name} failed on rank {rank}: {e!r}")
            extras.append({"workload": name, "error": repr(e)})
    if rank == 0:
        spec = WORKLOADS[args.workload]
        line = {
            "metric": "user-solve updates/sec + sec/epoch, "
                      f"{spec['model'].upper() if spec['model'] == 'safer2' else 'iALS'} "
                      f"dim={spec['dim']} {spec['shape']}-shaped",
            "value": head["value"],
            "unit": "user-solve updates/s",
            "n_gpus": world,
            "rccl_ranks": head["rccl_ranks"],
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"],
            "sec_per_epoch": head["sec_per_epoch"],
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic ({spec['shape']}-shaped, Zipf-Mandelbrot items, lognormal users, "
                    "seed 98765); random init seed 1",
            "config": {"workload": f"{head['workload']}: {spec['model']} d={spec['dim']} "
                                   f"{spec['shape']}-shaped synthetic, one Train() epoch per step "
                                   f"({spec['readme']} flags, print_train_stats 0)",
                       "n_users": head["n_users"], "n_items": head["n_items"],
                       "nnz": head["nnz"], "dim": head["dim"], "padded_dim": head["padded_dim"],
                       "flags": spec["flags"], "parallelism": f"entity-sharded x{world}"},
            "timed_path": "frecsys_model_train -> Recommender::Train (include/frecsys_model.h)",
            "frecsys_env": env,
        }
        for k in ("u_halfstep_solve_updates_per_s", "kernel_ms_per_epoch", "roofline", "paths",
                  "gather_roofline", "loss_gather_roofline", "cpu_baseline", "hspace_reruns",
                  "tagged_timeouts"):
            line[k] = head[k]
        line["workloads"] = {r["workload"]: r for r in extras}
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
