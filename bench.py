#!/usr/bin/env python3
"""Flagship benchmark: distributed Lloyd K-Means, N=10M points, D=128, K=1024, bf16.

Metric (BASELINE.json): points assigned / s (whole job) and iters / s of "K-Means N=10M
D=128 K=1024 at 1/2/4/8 MI355X".  One *step* is one full Lloyd iteration on every rank:
bf16 MFMA distance + fused argmin (HIP), LDS centroid update (HIP), ONE packed RCCL
all-reduce of [sums | counts], centroid finalize (HIP).  Nothing is skipped inside the
timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N

Warm-up: W steps, continued (untimed, same count on every rank) until the warm-up has run
``--settle-ms`` (250) on the GPU -- the clock ramps over the first ~50 ms of MFMA load --
then back to the init snapshot; the JSON's ``warmup`` is W, ``warmup_steps_run`` /
``warmup_ms`` what ran.

Data: synthetic Gaussian blobs generated on each GPU (counter-based, world-size
invariant), random-row centroid init.  The default ``headline`` preset is STRONG scaling:
N = 10M points in total, split over the ranks (1.25M rows per GPU at N=8), exactly the
BASELINE.json metric; ``headline_weak`` keeps 10M points per GPU.  ``--n-per-gpu`` is the
rows per GPU under ``--scaling weak`` and the TOTAL rows under ``--scaling strong``.  At
world > 1 the JSON carries ``phase_ms`` (assign / update / all-reduce / finalize device
time of one step, max over ranks).
``vs_baseline`` compares only like with like: it is set for the reference's own configs
(``--preset ref25m_kmeans`` / ``ref25m_fcm``: N=25M, D=5, K=3, fp64) against the
executions_log.csv row with the same method and GPU count, and is null otherwise -- the
reference never ran the BASELINE.json configs.  ``vs_reference_best``
always divides by the reference's best number for the method (K-Means 177.7 M points/s,
N=25M D=5 K=3 8 GPUs fp64, scripts/executions_log.csv:320; FCM 325.8 M, :321), the floor
BASELINE.md sets for the north-star configs.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

BASELINE_POINTS_PER_SEC = 177.7e6       # K-Means, scripts/executions_log.csv:320
BASELINE_FCM_POINTS_PER_SEC = 325.8e6   # FCM, scripts/executions_log.csv:321
# same-config rows (N=25M, D=5, K=3, fp64, 20 iters) by GPU count, points assigned/s
# (BASELINE.md full table; the 1-GPU runs and some FCM counts failed in the reference)
REF25M_K3 = {
    "kmeans": {2: 70.5e6, 3: 85.6e6, 4: 119.1e6, 5: 128.4e6, 6: 140.5e6, 7: 157.2e6, 8: 177.7e6},
    "fcm": {2: 93.2e6, 4: 178.4e6, 7: 291.5e6, 8: 325.8e6},
}

# BASELINE.json configs (the default is the headline metric/config)
PRESETS = {
    "headline": dict(n_per_gpu=10_000_000, dim=128, k=1024, scaling="strong", mode="lloyd"),
    "headline_weak": dict(n_per_gpu=10_000_000, dim=128, k=1024, scaling="weak", mode="lloyd"),
    "dp100m": dict(n_per_gpu=100_000_000, dim=128, k=1024, scaling="strong", mode="lloyd"),
    "minibatch1b": dict(n_per_gpu=1_000_000_000, dim=64, k=4096, scaling="strong",
                        mode="minibatch", batch_size=1 << 20),
    # the reference's published configs (scripts/executions_log.csv): N=25M, D=5, fp64
    "ref25m_kmeans": dict(n_per_gpu=25_000_000, dim=5, k=3, scaling="strong", mode="lloyd",
                          dtype="fp64"),
    "ref25m_fcm": dict(n_per_gpu=25_000_000, dim=5, k=3, scaling="strong", mode="lloyd",
                       dtype="fp64", method="fcm"),
    "embed50m_fp8": dict(n_per_gpu=50_000_000, dim=768, k=65536, scaling="strong", mode="lloyd",
                         dtype="fp8"),
    # FCM at the headline shape on the bf16 MFMA tower: bf16x3 distances in both passes
    # (the library default; --fcm-distances one: one product + two-nearest fix-up, ~20 %
    # faster but 4 % off in the centroids on this data, profiles/bench_fcm10m_one_std025_r06h),
    # fp32 memberships, bf16 weights x the bf16 rows in W^T X (ops.FCM_PRECISION, reported
    # with the witness; --dtype fp32 / fp64 run the fp64 matrix-core path), m = 2 (the
    # reference's m = D = 128 would underflow every u^m).
    # cluster_std 0.25: at the blob generator's default 1.0, m=2 FCM at D=128, K=1024 pulls
    # every centroid onto the grand mean within the timed steps (distance concentration;
    # the final-state witness was then vacuous, final_ws_spread 0.0); at 0.25 the clusters
    # keep their structure (tests/test_bench_cpu.py::test_fcm10m_preset_keeps_structure)
    "fcm10m": dict(n_per_gpu=10_000_000, dim=128, k=1024, scaling="weak", mode="lloyd",
                   dtype="bf16", method="fcm", fuzzifier=2.0, fcm_distances="x3",
                   cluster_std=0.25),
}


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n-per-gpu", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--dtype", default="bf16", choices=["fp8", "bf16", "fp32", "fp64"])
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="strong: --n-per-gpu is the total N split over the ranks; weak: "
                         "every rank owns --n-per-gpu rows")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cluster-std", type=float, default=1.0,
                    help="standard deviation of the synthetic Gaussian blobs (centres "
                         "uniform in [-10, 10]^D)")
    ap.add_argument("--preset", default="headline", choices=sorted(PRESETS),
                    help="BASELINE config: headline (N=10M total D=128 K=1024, strong "
                         "scaling, default), headline_weak (10M per GPU), "
                         "dp100m (N=100M total), minibatch1b (mini-batch N=1B D=64 K=4096), "
                         "embed50m_fp8 (N=50M D=768 K=65536, fp8 block-scaled MFMA), "
                         "ref25m_kmeans / ref25m_fcm (the reference's own N=25M D=5 K=3 fp64)")
    ap.add_argument("--batch-size", type=int, default=0, help="mini-batch rows per rank")
    ap.add_argument("--method", default="kmeans", choices=["kmeans", "fcm"],
                    help="fcm: distributed Fuzzy C-Means step (fuzzifier m = D, as the reference)")
    ap.add_argument("--init", default="random", choices=["random", "kmeans++", "kmeans||", "first_k"],
                    help="centroid init (timed separately as init_s; the north star's random "
                         "rows by default; kmeans++ switches to sampled k-means|| above K=2048)")
    ap.add_argument("--fuzzifier", type=float, default=None,
                    help="FCM fuzzifier m (default: the reference's m = D)")
    ap.add_argument("--algorithm", default="lloyd", choices=["lloyd", "bounded"],
                    help="bounded: Lloyd with Hamerly bounds (not the headline metric's "
                         "algorithm; reported in config.algorithm)")
    ap.add_argument("--source", default="device", choices=["device", "host"],
                    help="host: the shard lives in host memory (fp32) and streams through "
                         "HBM via the native RowStreamer (pinned ring + copy stream), with "
                         "the hybrid-residency planner under --hbm-budget-gb")
    ap.add_argument("--hbm-budget-gb", type=float, default=0.0,
                    help="per-GPU HBM budget of the stream planner (--source host)")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step from a captured HIP graph (1 GPU; RCCL capture for N>1)")
    ap.add_argument("--profile-steps", action="store_true",
                    help="add a per-phase breakdown (phase_ms) after the timed region "
                         "(always on at world > 1)")
    ap.add_argument("--centers-out", default=None,
                    help="rank 0 writes the final centroids (.npy, fp64) here")
    ap.add_argument("--update", default="auto", choices=["auto", "full", "delta"],
                    help="K-Means centroid update: delta moves only the rows whose label "
                         "changed between fp64 running totals (with a full re-sum every "
                         "--delta-refresh steps and after steps that moved > 40%% of the rows); "
                         "full re-sums every row every step; auto = delta where supported")
    ap.add_argument("--fcm-distances", default="x3", choices=["one", "x3"],
                    help="bf16 FCM distances: one product + two-nearest fix-up, or bf16x3 "
                         "(ClusterConfig.fcm_distances)")
    ap.add_argument("--fcm-path", default="", choices=["", "tower", "wide", "wide64"],
                    help="FCM A/B: force the SIMT tower, the wide path, or the fp64 matrix-core "
                         "path for any dtype (ops.FCM_FORCE_PATH; default: the measured routing)")
    ap.add_argument("--settle-ms", type=float, default=None,
                    help="after the W warm-up steps keep stepping (untimed) until the warm-up "
                         "has run this many ms, so the timed steps start at the settled GPU "
                         "clock (it ramps over the first ~50 ms of MFMA load); default 250 on "
                         "a GPU, 0 on the CPU; 0 = exactly W warm-up steps")
    ap.add_argument("--fp8-recheck", type=float, default=0.0,
                    help="fp8 K-Means: exact re-check of rows whose fp8 margin to the runner-up "
                         "is within this relative tau (ClusterConfig.fp8_recheck; 0 = off)")
    ap.add_argument("--no-x3-prefilter", action="store_true",
                    help="fp32/fp64 K-Means: run the bf16x3 pass over every row (no one-product "
                         "prefilter; A/B of HipX3Lloyd.prefilter)")
    ap.add_argument("--x3-full-grid", action="store_true",
                    help="fp32/fp64 K-Means: size the listed bf16x3 launch by N instead of the "
                         "last listed share (A/B of HipX3Lloyd.listed_estimate)")
    ap.add_argument("--comm-mode", default="auto", choices=["auto", "allreduce", "rsag"],
                    help="partial-sum reduction (ClusterConfig.comm_mode); with "
                         "TDC_FORCE_COLLECTIVES=1 a world-1 run issues the RCCL calls too")
    ap.add_argument("--delta-refresh", type=int, default=32,
                    help="delta update: full re-sum every this many steps (0: never)")
    ap.add_argument("--deterministic", action="store_true",
                    help="bitwise reproducible update (int64 fixed-point partial sums)")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the correctness witness after the timed region")
    ap.add_argument("--warm-start", action="store_true",
                    help="time the K steps right after the warm-up steps (the round-4 protocol) "
                         "instead of rewinding to the centroid init")
    ap.add_argument("--no-steady", action="store_true",
                    help="skip the second (steady-state) window after the timed one")
    a = ap.parse_args(argv)
    p = PRESETS[a.preset]
    given = set(x.split("=")[0].lstrip("-").replace("-", "_") for x in (argv or sys.argv[1:]))
    for key, val in p.items():
        if key not in given:
            setattr(a, key, val)
    return a


def main(argv=None):
    a = parse(argv)
    import torch
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
    from tensorflow_distributed_clustering_amd.models.kmeans import LloydEngine
    from tensorflow_distributed_clustering_amd.parallel.dist import init_comm, shard_bounds

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != a.gpus and world_env > 1:
        print(f"[bench] warning: WORLD_SIZE={world_env} but --gpus={a.gpus}", file=sys.stderr)
    if a.gpus > 1 and world_env == 1:
        # self-launch one process per GPU (before touching the GPU in this process)
        import subprocess
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={a.gpus}", "--master-addr=127.0.0.1",
               f"--master-port={29500 + (os.getpid() % 1000)}", os.path.abspath(__file__)] + \
              (sys.argv[1:] if argv is None else list(argv))
        sys.exit(subprocess.call(cmd))

    if a.fcm_path:
        import tensorflow_distributed_clustering_amd.ops as _ops
        _ops.FCM_FORCE_PATH = a.fcm_path
    comm = init_comm("cuda" if torch.cuda.is_available() else "cpu")
    dev = comm.device
    world, rank = comm.world_size, comm.rank
    n_global = a.n_per_gpu * world if a.scaling == "weak" else a.n_per_gpu
    s, e = shard_bounds(n_global, world, rank)
    dt = {"fp8": torch.bfloat16, "bf16": torch.bfloat16, "fp32": torch.float32,
          "fp64": torch.float64}[a.dtype]
    src_info = None
    if a.source == "host":
        x, src_info = host_shard(a, e - s, s, dev, torch)
    else:
        x = gaussian_blobs(e - s, a.dim, a.k, seed=a.seed, row_offset=s, dtype=dt, device=dev,
                           cluster_std=a.cluster_std)
    cfg = tdc.ClusterConfig(n_clusters=a.k, max_iter=a.steps, dtype=a.dtype, init=a.init,
                            seed=a.seed, compute_inertia=False, algorithm=a.algorithm,
                            fuzzifier=a.fuzzifier, update=a.update,
                            delta_refresh=a.delta_refresh, deterministic=a.deterministic,
                            comm_mode=a.comm_mode, fcm_distances=a.fcm_distances,
                            fp8_recheck=a.fp8_recheck)
    if a.mode == "minibatch":
        from tensorflow_distributed_clustering_amd.models.minibatch import MiniBatchStepper
        eng = MiniBatchStepper(x, cfg.replace(batch_size=a.batch_size or (1 << 20)), comm,
                               n_global, s)
        points_per_step = eng.batch_rows * world
    elif a.method == "fcm":
        from tensorflow_distributed_clustering_amd.models.fcm import FcmEngine
        eng = FcmEngine(x, cfg, comm, n_global, s, defer_init=True)
        points_per_step = n_global
    elif a.algorithm == "bounded":
        from tensorflow_distributed_clustering_amd.models.bounded import BoundedLloydEngine
        eng = BoundedLloydEngine(x, cfg, comm, n_global, s, defer_init=True)
        points_per_step = n_global
    else:
        if src_info is not None:
            eng = LloydEngine(x, cfg, comm, n_global, s, chunk_rows=src_info["chunk_rows"],
                              defer_init=True)
        else:
            eng = LloydEngine(x, cfg, comm, n_global, s, defer_init=True)
        points_per_step = n_global
    if a.no_x3_prefilter and hasattr(getattr(eng, "local", None), "prefilter"):
        eng.local.prefilter = False
    if a.x3_full_grid and hasattr(getattr(eng, "local", None), "listed_estimate"):
        eng.local.listed_estimate = False
    init_s = None
    if hasattr(eng, "init_centroids") and getattr(eng, "c0", None) is None:
        # the centroid init, timed on its own (never inside the timed steps)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        t_i = time.perf_counter()
        eng.init_centroids()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        init_s = comm.max_scalar(time.perf_counter() - t_i)
    graph = False
    if a.mode == "lloyd" and a.method == "kmeans" and a.algorithm == "lloyd" and a.graph \
            and dev.type == "cuda":
        eng.capture(include_collectives=comm.collective)
        graph = True

    # warm-up steps (code objects, grid sizing, RCCL communicators), then back to the
    # init: the timed steps are iterations 1..K from the centroid init, as the reference's
    # computation_time (scripts/distribuitedClustering.py:277-280) -- the high-motion
    # first iterations and the delta update's first full step are inside the window
    snap = eng.snapshot() if (hasattr(eng, "snapshot") and not a.warm_start) else None
    t_w = time.perf_counter()
    for _ in range(a.warmup):
        eng.step()
    warm_steps = a.warmup
    # clock settle: the GPU raises its clock over the first ~50 ms of sustained MFMA load
    # (the headline assign runs 2.1-2.4 ms per call at first and 1.81 ms from ~50 ms on,
    # profiles/clock_ramp_r06w.txt), so W short warm-up steps would leave the timed steps
    # inside the ramp.  The warm-up keeps stepping, untimed, until it has run --settle-ms;
    # every rank runs the same number of steps (one flag all-reduce per extra step); the
    # timed steps still start from the init snapshot below
    settle_ms = a.settle_ms if a.settle_ms is not None else (250.0 if dev.type == "cuda" else 0.0)
    while a.warmup > 0 and settle_ms > 0 and warm_steps < 20000:
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        short = (time.perf_counter() - t_w) * 1e3 < settle_ms
        if comm.max_scalar(1.0 if short else 0.0) == 0.0:
            break
        eng.step()
        warm_steps += 1
    warm_ms = (time.perf_counter() - t_w) * 1e3
    if snap is not None:
        eng.rewind(snap)

    def timed(nsteps):
        comm.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        u0 = eng.update_stats() if hasattr(eng, "update_stats") else None
        t_0 = time.perf_counter()
        for _ in range(nsteps):
            eng.step()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        comm.barrier()
        el = comm.max_scalar(time.perf_counter() - t_0)
        u1 = eng.update_stats() if hasattr(eng, "update_stats") else None
        info = None
        if u0 is not None and u1 is not None:
            dm = u1["moved_rows"] - u0["moved_rows"]
            ds = u1["moved_steps"] - u0["moved_steps"]
            info = {"moved_frac_mean": dm / max(1.0, ds) / max(1, n_global),
                    "full_steps_timed": int(u1["full_steps"] - u0["full_steps"])}
        return el, info

    h2d0 = getattr(x, "bytes_h2d", 0) if src_info is not None else 0
    elapsed, upd_init = timed(a.steps)
    if src_info is not None:
        src_info["h2d_GBps"] = (x.bytes_h2d - h2d0) / elapsed / 1e9

    ms = elapsed / max(1, a.steps) * 1e3
    pps = points_per_step * a.steps / elapsed
    # ---- everything below runs after the timed region ----
    # steady state: the next K iterations (the clustering has converged most of the way),
    # reported beside the from-init number, never instead of it
    ms_steady, upd_steady = None, None
    if snap is not None and not a.no_steady and elapsed * 2 < 120.0:
        el_s, upd_steady = timed(a.steps)
        ms_steady = el_s / max(1, a.steps) * 1e3
    update_info = None
    if hasattr(eng, "update_stats"):
        update_info = {"mode": eng.update_mode, "refresh_every": a.delta_refresh}
        if upd_init is not None:
            update_info.update(upd_init)
        if upd_steady is not None:
            update_info["steady"] = upd_steady
    check = None
    if not a.no_check and src_info is None:
        if a.method == "fcm":
            check = fcm_witness(eng, x, n_global, s, e, comm, torch, a,
                                C0=snap["C"] if snap is not None else None)
        else:
            check = witness(eng, x, n_global, s, e, comm, torch, a)
    breakdown = None
    if ((a.profile_steps or world > 1) and a.mode == "lloyd" and a.method == "kmeans"
            and a.algorithm == "lloyd" and not getattr(eng, "streamed", False)):
        breakdown = phase_breakdown(eng, torch, dev)
    if a.centers_out:
        c = eng.centers() if hasattr(eng, "centers") else eng.C
        if rank == 0:
            import numpy as np
            np.save(a.centers_out, c.double().cpu().numpy())
    if rank == 0:
        out = {
            "metric": "points_assigned_per_sec",
            "value": pps,
            "unit": "points/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "warmup_steps_run": warm_steps,
            "warmup_ms": warm_ms,
            "ms_per_step": ms,
            "timed_from": "warm" if snap is None else "init",
            "ms_per_step_steady": ms_steady,
            "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": vs_baseline(a, world, pps),
            "vs_reference_best": pps / (BASELINE_FCM_POINTS_PER_SEC if a.method == "fcm"
                                        else BASELINE_POINTS_PER_SEC),
            "dtype": a.dtype,
            "precision": precision_of(eng, a),
            "data": "synthetic gaussian blobs (on-device, counter-based, std "
                    f"{a.cluster_std:g}), random-row init",
            "preset": a.preset,
            "init": {"method": a.init, "seconds": init_s},
            "iters_per_sec": 1e3 / ms,
            "backend": eng.local.name,
            "config": {"model": ("kmeans-minibatch" if a.mode == "minibatch" else
                                 "fuzzy-cmeans" if a.method == "fcm" else "kmeans-lloyd"),
                       "global_batch": points_per_step, "seq_len": a.dim, "N": n_global,
                       "K": a.k, "D": a.dim, "points_per_gpu": e - s,
                       "parallelism": f"dp{world}"},
        }
        if update_info is not None:
            out["update"] = update_info
        out["comm"] = {"mode": "rsag" if getattr(eng, "rsag", False) else "allreduce",
                       "collective": bool(comm.collective), "backend": comm.backend}
        out["graph_replay"] = graph
        if check is not None:
            out["check"] = check
        if breakdown:
            out["phase_ms"] = breakdown
        if src_info is not None:
            out["data"] = "synthetic gaussian blobs in HOST memory (fp32), streamed via RowStreamer"
            out["source"] = src_info
        if a.algorithm != "lloyd":
            out["config"]["algorithm"] = a.algorithm
        if a.deterministic:
            out["config"]["deterministic"] = True
        if a.fp8_recheck:
            out["config"]["fp8_recheck"] = a.fp8_recheck
        if a.method == "fcm":
            out["config"]["fuzzifier"] = a.fuzzifier if a.fuzzifier is not None else a.dim
            out["active_frac_last_step"] = getattr(eng, "active_frac", None)
        print(json.dumps(out), flush=True)
    from tensorflow_distributed_clustering_amd.parallel.dist import destroy_comm
    destroy_comm()  # a clean process-group teardown (RCCL warns otherwise)


def host_shard(a, n_rows, row_offset, dev, torch):
    """The rank's shard generated in host memory (fp32) and wrapped in a HostSource with the
    hybrid-residency planner: the first rows that fit the budget stay in HBM, the rest
    streams every pass (RowStreamer threads convert to the kernel layout into a pinned
    ring; H2D on a copy stream)."""
    import numpy as np
    from tensorflow_distributed_clustering_amd.data.stream import (HostSource, plan_chunk_rows,
                                                                   plan_resident_rows)
    from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
    from tensorflow_distributed_clustering_amd.ops import padded_dim
    xh = np.empty((n_rows, a.dim), dtype=np.float32)
    step = 1 << 24
    t0 = time.perf_counter()
    for r0 in range(0, n_rows, step):
        r1 = min(n_rows, r0 + step)
        xh[r0:r1] = gaussian_blobs(r1 - r0, a.dim, a.k, seed=a.seed, row_offset=row_offset + r0,
                                   dtype=torch.float32, device=dev).cpu().numpy()
        if (r0 // step) % 8 == 0:
            print(f"[bench] host shard {r1}/{n_rows} rows ({time.perf_counter() - t0:.0f} s)",
                  file=sys.stderr, flush=True)
    width = padded_dim(a.dim) if a.dtype == "bf16" else a.dim
    es = 2 if a.dtype == "bf16" else 4
    layout = (torch.bfloat16 if a.dtype == "bf16" else torch.float32, width)
    chunk = a.batch_size if a.mode == "minibatch" and a.batch_size else \
        (plan_chunk_rows(n_rows, width * es, a.k, a.dim, dev, a.hbm_budget_gb) or (1 << 22))
    resident = plan_resident_rows(n_rows, width * es, chunk, a.k, a.dim, dev, a.hbm_budget_gb)
    src = HostSource(xh, layout, dev, row_offset, resident_rows=resident, n_threads=16)
    return src, {"rows": n_rows, "resident_rows": resident, "chunk_rows": chunk,
                 "hbm_budget_gb": a.hbm_budget_gb}


def precision_of(eng, a):
    """What the timed step computes, in words (the dtype key alone undersells fp32 on the
    matrix cores and oversells the MFMA FCM tower)."""
    name = getattr(getattr(eng, "local", None), "name", "")
    if a.method == "fcm":
        from tensorflow_distributed_clustering_amd.ops import FCM_PRECISION
        own = getattr(getattr(eng, "local", None), "precision", None)
        if isinstance(own, str):
            return own
        return FCM_PRECISION.get(getattr(eng, "dtype_name", a.dtype), a.dtype)
    if name == "hip_x3_mfma":
        pre = ("one-product bf16 MFMA prefilter certifying rows by its own bound, then "
               if getattr(eng.local, "pre", None) is not None and eng.local.prefilter else "")
        return (f"{a.dtype} exact-argmin labels: {pre}bf16x3 MFMA scores + exact {a.dtype} "
                f"re-check of the rows the error bound cannot certify; {a.dtype} rows in the update")
    if a.dtype == "fp8":
        return "fp8 e4m3 block-scaled MFMA distances; sums from the bf16 rows"
    if a.dtype == "bf16":
        return "bf16 MFMA distances (fp32 accumulate); sums of the bf16 rows in fp32/fp64"
    return f"{a.dtype} difference-form distances"


def vs_baseline(a, world, pps):
    """value / the reference's number for the SAME config and GPU count, else None."""
    same = (a.n_per_gpu == 25_000_000 and a.scaling == "strong" and a.dim == 5 and a.k == 3
            and a.dtype == "fp64" and a.mode == "lloyd")
    ref = REF25M_K3["fcm" if a.method == "fcm" else "kmeans"].get(world) if same else None
    return pps / ref if ref else None


def phase_breakdown(eng, torch, dev, reps: int = 5):
    """Per-phase time of one step, max over ranks (diagnostic, after the timed run; the
    phases (``LloydEngine.phase_fns``: buffer fill, assign, local update -- the delta update
    when the engine uses it --, all-reduce, finalize) run eagerly with an event -- or a host
    clock on CPU -- between them, so their sum is a little above a graph-replayed step).
    The all-reduce phase includes the wait for the slowest rank.  rsag engines:
    "allreduce" is reduce-scatter + all-gather + the slice finalize, "finalize" is empty."""
    cuda = dev.type == "cuda"
    phases = eng.phase_fns()
    if getattr(eng, "rsag", False):
        phases = phases[:3] + [("allreduce", eng._reduce_scatter_finalize),
                               ("finalize", lambda: None)]
    names = [n for n, _ in phases]
    tot = {n: 0.0 for n in names}
    c_keep = eng.C.clone()
    eng.comm.barrier()
    for _ in range(reps):
        e, t = [], []

        def rec():
            ev = torch.cuda.Event(enable_timing=True) if cuda else None
            if ev is not None:
                ev.record()
            e.append(ev)
            t.append(time.perf_counter())
        rec()
        for _, fn in phases:
            fn()
            rec()
        if cuda:
            torch.cuda.synchronize(dev)
        for i, n in enumerate(names):
            dt = e[i].elapsed_time(e[i + 1]) if cuda else (t[i + 1] - t[i]) * 1e3
            tot[n] += dt / reps
    eng.C.copy_(c_keep)  # leave the engine's centroids as the timed run left them
    eng.local.prepare(eng.C)
    vals = torch.tensor([tot[n] for n in names], dtype=torch.float64, device=dev)
    eng.comm.allreduce_(vals, "max")
    return {n: round(float(v), 4) for n, v in zip(names, vals.tolist())}


WITNESS_ROWS = 65536


def fcm_witness(eng, x, n_global, s, e, comm, torch, a, C0=None):
    """FCM correctness witness, after the timed region: ONE FCM step on a fixed sample of
    WITNESS_ROWS global rows (evenly spaced, world-size invariant), computed by the same
    native tower the engine runs and by the fp64 oracle (plain PyTorch difference-form
    distances, `scripts/distribuitedClustering.py:112-137`); reported: the centroid error
    max|c - c_ref| / max|c_ref| and the worst relative error of sum_i w_ik over the
    clusters holding >= 1e-6 of the total weight -- from the final centroids, and (key
    ``at_init``) from the init centroids C0.  FCM at m = 2 on well-mixed high-D data can
    collapse every centroid onto the grand mean (distance concentration: u -> 1/K); the
    final step is then trivially exact (w = K^-2 is a bf16 number), which
    ``final_ws_spread`` = (max - min) / mean of sum_i w_ik shows, while the init step keeps
    the memberships spread."""
    from tensorflow_distributed_clustering_amd.ops import FCM_PRECISION, make_fcm_ops
    from tensorflow_distributed_clustering_amd.ops import reference as ref
    dev = comm.device
    g = torch.arange(WITNESS_ROWS, dtype=torch.float64) * (n_global / WITNESS_ROWS)
    g = torch.unique(g.floor().long())
    loc = (g[(g >= s) & (g < e)] - s).to(dev)
    nz = eng.cfg.fcm_nan_to_zero

    def at(C):
        C = C.double()
        k, d = C.shape
        xs = x.index_select(0, loc)[:, :d] if loc.numel() else x[:0, :d]
        wx = torch.zeros(k, d, dtype=torch.float64, device=dev)
        ws = torch.zeros(k, dtype=torch.float64, device=dev)
        wr = torch.zeros(k, d, dtype=torch.float64, device=dev)
        wsr = torch.zeros(k, dtype=torch.float64, device=dev)
        ops = None
        if xs.shape[0]:
            # the engine's own operand dtype: a bf16 shard reaches the tower as bf16
            xin = xs.double() if eng.dtype_name == "fp64" else (
                xs if xs.dtype == torch.bfloat16 else xs.float())
            ops = make_fcm_ops(xin, k, eng.dtype_name, eng.m, nz, eng.cfg.backend,
                               eng.cfg.fcm_distances)
            lab = torch.empty(xs.shape[0], dtype=torch.int32, device=dev)
            ops.step(C.to(ops.c_dtype).contiguous(), lab, wx, ws)
            step = max(1, (1 << 24) // max(1, k * d))
            for r0 in range(0, xs.shape[0], step):
                # exact difference form: a sampled row that IS a centroid (random-row init)
                # is at distance exactly 0, the rule the native towers apply
                pa, pb, _ = ref.fcm_partial(xs[r0:r0 + step].double(), C, eng.m, nz,
                                            acc_dtype=torch.float64, exact=True)
                wr += pa
                wsr += pb
        for t in (wx, ws, wr, wsr):
            comm.allreduce_(t)
        c_k = wx / ws.clamp_min(1e-300)[:, None]
        c_r = wr / wsr.clamp_min(1e-300)[:, None]
        ok = wsr > 1e-6 * float(wsr.sum())
        cerr = float((c_k - c_r)[ok].abs().max()) / max(1e-300, float(c_r[ok].abs().max())) \
            if bool(ok.any()) else 0.0
        werr = float(((ws - wsr).abs() / wsr.clamp_min(1e-300))[ok].max()) \
            if bool(ok.any()) else 0.0
        spread = float((wsr.max() - wsr.min()) / wsr.mean().clamp_min(1e-300))
        return {"fcm_centroid_rel_err": cerr, "fcm_weight_sum_rel_err": werr,
                "ws_spread": spread,
                "precision": (getattr(ops, "precision", None) if ops is not None else None)
                or FCM_PRECISION.get(eng.dtype_name, eng.dtype_name),
                "backend": ops.name if ops is not None else None}

    out = at(eng.centers())
    out["final_ws_spread"] = out.pop("ws_spread")
    out["sample_rows"] = int(comm.sum_scalar(float(loc.numel())))
    if C0 is not None:
        ini = at(C0)
        out["at_init"] = {kk: ini[kk] for kk in ("fcm_centroid_rel_err",
                                                 "fcm_weight_sum_rel_err", "ws_spread")}
    return out


def witness(eng, x, n_global, s, e, comm, torch, a):
    """Correctness witness, computed after the timed region (never inside it): a label pass
    against the final centroids, then (1) the global inertia sum_i ||x_i - c_{label_i}||^2
    in fp64 over every row, and (2) the agreement of the kernel labels with an exact fp64
    argmin on a fixed sample of WITNESS_ROWS global rows (evenly spaced,
    world-size invariant).  The oracle sees the same rows the kernels see (the bf16 shard
    upcast), so disagreements are near ties of the bf16 / fp8 distance arithmetic;
    ``agree_tie_tol`` also counts a label whose exact distance is within 1e-5 (relative)
    of the exact minimum, and ``agree_fp64_kernel_operands`` the agreement with the fp64
    argmin over the operands the kernels use (bf16-rounded centroids on the bf16 paths):
    the bf16 centroid rounding, not the kernel arithmetic, is what separates the first
    number from 1."""
    from tensorflow_distributed_clustering_amd.ops import reference as ref
    dev = comm.device
    C = (eng.centers() if hasattr(eng, "centers") else eng.C).double()
    if hasattr(eng, "blabels"):  # mini-batch stepper: labels from its own label pass
        labels, _ = eng.label_pass()
    else:
        eng.label_pass()
        labels = eng.labels
    xs = x[:, : C.shape[1]]
    inertia = 0.0
    step = max(1, (1 << 26) // max(1, C.shape[1]))
    for r0 in range(0, xs.shape[0], step):
        r1 = min(xs.shape[0], r0 + step)
        diff = xs[r0:r1].double() - C.index_select(0, labels[r0:r1].long())
        inertia += float(diff.pow_(2).sum())
    g = torch.arange(WITNESS_ROWS, dtype=torch.float64) * (n_global / WITNESS_ROWS)
    g = torch.unique(g.floor().long())
    loc = g[(g >= s) & (g < e)] - s
    agree = near = agree_op = 0.0
    # the centroids as the assignment kernels see them: bf16 MFMA paths round them to bf16
    # (fp8 quantises rows and centroids block-wise: no simple operand oracle, not reported)
    c_op = C.to(torch.bfloat16).double() if a.dtype == "bf16" and a.method == "kmeans" else C
    if loc.numel():
        idx = loc.to(dev)
        xsm = xs.index_select(0, idx).double()
        lab_o, d_o = ref.assign(xsm, C, exact=False)  # fp64 GEMM form
        lab_k = labels.index_select(0, idx).long()
        d_k = (xsm - C.index_select(0, lab_k)).pow_(2).sum(1)
        agree = float((lab_o.long() == lab_k).sum())
        near = float((d_k <= d_o.double() * (1 + 1e-5) + 1e-12).sum())
        lab_p, _ = ref.assign(xsm, c_op, exact=False)
        agree_op = float((lab_p.long() == lab_k).sum())
    tot = comm.sum_scalar(float(loc.numel()))
    out = {"inertia": comm.sum_scalar(inertia),
           "agree_fp64_sample": comm.sum_scalar(agree) / max(1.0, tot),
           "agree_tie_tol": comm.sum_scalar(near) / max(1.0, tot),
           "sample_rows": int(tot)}
    amb = getattr(eng.local, "ambiguous_rows", None)
    if amb is not None:
        # fp32/fp64 MFMA path: rows of the last label pass re-checked exactly
        out["recheck_rows_frac"] = comm.sum_scalar(float(amb())) / max(1, n_global)
        out["rescan_rows_frac"] = comm.sum_scalar(float(eng.local.rescanned_rows())) / max(1, n_global)
        # rows the one-product prefilter could not certify (the three-product pass's share)
        out["x3_rows_frac"] = comm.sum_scalar(float(eng.local.prefilter_rows())) / max(1, n_global)
    if a.dtype != "fp8":
        # fp64 argmin over the kernel's own operands (bf16 rows, bf16-rounded centroids)
        out["agree_fp64_kernel_operands"] = comm.sum_scalar(agree_op) / max(1.0, tot)
    else:
        comm.sum_scalar(agree_op)  # every rank issues the same collectives
    return out


if __name__ == "__main__":
    main()
