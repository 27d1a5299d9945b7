"""Data-parallel correctness without GPUs: world sizes 2/3/4 on the gloo backend must
reproduce the single-process result (fp64; equal up to the summation order of the
packed all-reduce).  Replaces the reference's lack of any fake-cluster testing.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, method, init, q, n, d, k, iters, seed, extra):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
    from tensorflow_distributed_clustering_amd.parallel import dist as D
    D._COMM = None
    comm = D.init_comm("cpu")
    s, e = comm.shard(n)
    x = gaussian_blobs(e - s, d, k, seed=seed, row_offset=s, dtype=torch.float64)
    kw = dict(n_clusters=k, max_iter=iters, dtype="fp64", init=init, seed=seed)
    kw.update(extra)
    cfg = tdc.ClusterConfig(**kw)
    model = (tdc.KMeans if method == "kmeans" else tdc.FuzzyCMeans)(cfg, comm)
    model.fit(x, n_global=n, row_offset=s)
    r = model.result_
    labels = comm.gather_rows_to_root(r.labels)
    info = {}
    eng = getattr(model, "engine_", None)
    if eng is not None:
        info = dict(rsag=getattr(eng, "rsag", False), split=getattr(eng, "count_split", False),
                    counts=r.counts, update_mode=getattr(eng, "update_mode", None),
                    update_stats=eng.update_stats() if hasattr(eng, "update_stats") else None)
    if rank == 0:
        q.put((r.centers, labels.numpy(), r.inertia, r.n_iter, r.init_centers, info))
    D.destroy_comm()


def run_world(world, method="kmeans", init="random", n=6001, d=3, k=5, iters=6, seed=11, extra=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, method, init, q, n, d, k, iters,
                                                seed, extra or {}))
             for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return out


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("init", ["random", "kmeans++"])
def test_kmeans_dp_equals_single(world, init):
    c1, l1, in1, it1, i1, _ = run_world(1, init=init)
    cw, lw, inw, itw, iw, _ = run_world(world, init=init)
    np.testing.assert_array_equal(i1, iw)  # init is world-size invariant
    np.testing.assert_allclose(cw, c1, rtol=1e-12, atol=1e-12)
    np.testing.assert_array_equal(lw, l1)
    assert abs(inw - in1) <= 1e-9 * abs(in1)
    assert itw == it1


def test_kmeans_parallel_init_world_invariant():
    c1, l1, in1, it1, i1, _ = run_world(1, init="kmeans||", k=8)
    c2, l2, in2, it2, i2, _ = run_world(2, init="kmeans||", k=8)
    np.testing.assert_allclose(i2, i1, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(c2, c1, rtol=1e-10, atol=1e-10)


def test_fcm_dp_equals_single():
    c1, l1, *_ = run_world(1, method="fcm", init="first_k", d=4, k=3)
    c4, l4, *_ = run_world(4, method="fcm", init="first_k", d=4, k=3)
    np.testing.assert_allclose(c4, c1, rtol=1e-12, atol=1e-12)
    np.testing.assert_array_equal(l4, l1)


def test_dp_tolerance_stop_consistent():
    c1, _, _, it1, _, _ = run_world(1, iters=200, extra={"tol": 1e-10})
    c2, _, _, it2, _, _ = run_world(2, iters=200, extra={"tol": 1e-10})
    assert it1 == it2 and it1 < 200
    np.testing.assert_allclose(c2, c1, rtol=1e-12, atol=1e-12)


# ---------------------------------------------------------------- collective layer
# every reduction branch of LloydEngine (SURVEY §5.8 / scripts/distribuitedClustering.py:
# 139-148,253-263, the reference's CPU add_n): one all-reduce, forced-small buckets,
# reduce-scatter -> sliced finalize -> all-gather (K not a multiple of the world size),
# and the exact fp32 count halves -- each equal to the single-rank fit
@pytest.mark.parametrize("world,extra", [
    (2, {"comm_mode": "allreduce"}),
    (3, {"comm_mode": "allreduce", "bucket_kb": 1}),
    (2, {"comm_mode": "rsag"}),
    (3, {"comm_mode": "rsag", "empty_cluster": "nan_any"}),
    (4, {"comm_mode": "rsag", "tol": 1e-12, "log_every": 2}),
])
def test_reduction_modes_equal_single(world, extra):
    kw = dict(k=7, d=5, iters=5)
    c1, l1, in1, it1, _, _ = run_world(1, extra=extra, **kw)
    cw, lw, inw, itw, _, info = run_world(world, extra=extra, **kw)
    assert info["rsag"] == (extra["comm_mode"] == "rsag")
    np.testing.assert_allclose(cw, c1, rtol=1e-12, atol=1e-12)
    np.testing.assert_array_equal(lw, l1)
    assert itw == it1


@pytest.mark.parametrize("world,mode", [(1, "allreduce"), (2, "allreduce"), (3, "rsag")])
def test_fp32_buffer_exact_counts(world, mode):
    # K*(D+1) > 65536: fp32 partial sums, counts ride as exact integer halves
    kw = dict(k=520, d=127, n=4001, iters=2)
    c, lab, _, _, _, info = run_world(world, extra={"dtype": "fp32", "comm_mode": mode}, **kw)
    assert info["split"] and info["rsag"] == (mode == "rsag")
    # counts of the last update = histogram of the labels it assigned (the final label
    # pass reassigns against the updated centroids, so compare totals only)
    assert info["counts"].sum() == kw["n"]
    assert np.all(info["counts"] == np.round(info["counts"]))
    c1, *_ = run_world(1, extra={"dtype": "fp32"}, **kw)
    np.testing.assert_allclose(c, c1, rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("world", [1, 2, 3])
def test_delta_update_equals_full(world):
    """update='delta' (only the rows whose label changed move between replicated fp64
    totals; full re-sum every 4 steps) reaches the full update's fit at every world size,
    and the ranks agree on every step's mode (the moved count rides in the all-reduce)."""
    kw = dict(k=9, d=4, n=9001, iters=14, init="first_k")
    cf, lf, inf_, itf, _, f = run_world(world, extra={"update": "full"}, **kw)
    cd, ld, ind, itd, _, dlt = run_world(world, extra={"update": "delta", "delta_refresh": 4},
                                         **kw)
    assert f["update_mode"] == "full" and dlt["update_mode"] == "delta"
    st = dlt["update_stats"]
    assert st["steps"] == 14 and st["full_steps"] == 1 + 13 // 4, st
    np.testing.assert_allclose(cd, cf, rtol=1e-10, atol=1e-10)
    np.testing.assert_array_equal(ld, lf)
    assert abs(ind - inf_) <= 1e-9 * abs(inf_) and itd == itf
    np.testing.assert_array_equal(dlt["counts"], f["counts"])


@pytest.mark.parametrize("world", [1, 2])
def test_delta_theta_fallback(world):
    """theta = 0: any step that moved a row makes the next one a full step (decided from
    the all-reduced moved count, so every rank switches together); same fit."""
    kw = dict(k=6, d=3, n=6007, iters=8)
    cf, lf, *_ = run_world(world, extra={"update": "full"}, **kw)
    cd, ld, _, _, _, info = run_world(world, extra={"update": "delta", "delta_theta": 0.0,
                                                    "delta_refresh": 0}, **kw)
    st = info["update_stats"]
    assert st["full_steps"] >= 2 and st["moved_rows"] > 0
    np.testing.assert_allclose(cd, cf, rtol=1e-10, atol=1e-10)
    np.testing.assert_array_equal(ld, lf)


@pytest.mark.parametrize("world,k,extra", [
    (2, 9, {"delta_refresh": 3}),
    (3, 7, {"delta_refresh": 3}),
    (3, 2, {"delta_refresh": 3}),  # the last rank's slice is all padding rows
    (2, 6, {"delta_refresh": 0, "delta_theta": 0.0}),
])
def test_delta_under_rsag_equals_full(world, k, extra):
    """Reduce-scatter mode keeps the delta update: each rank holds the fp64 totals of its
    own slice of centroid rows, the moved count and the signed count deltas ride in the
    all-reduced tail (every rank switches between delta and full steps together), and
    the fit equals the full update's under rsag and the single-rank fit."""
    kw = dict(k=k, d=4, n=9001, iters=10, init="first_k")
    cf, lf, inf_, itf, _, f = run_world(world, extra={"update": "full", "comm_mode": "rsag"}, **kw)
    cd, ld, ind, itd, _, dlt = run_world(world, extra=dict(update="delta", comm_mode="rsag",
                                                           **extra), **kw)
    assert dlt["rsag"] and dlt["update_mode"] == "delta" and f["update_mode"] == "full"
    st = dlt["update_stats"]
    if extra["delta_refresh"] == 3:
        assert st["steps"] == 10 and st["full_steps"] == 1 + 9 // 3, st
    else:
        assert st["full_steps"] >= 2 and st["moved_rows"] > 0, st
    np.testing.assert_allclose(cd, cf, rtol=1e-10, atol=1e-10)
    np.testing.assert_array_equal(ld, lf)
    np.testing.assert_array_equal(dlt["counts"], f["counts"])
    c1, l1, *_ = run_world(1, extra={"update": "full"}, **kw)
    np.testing.assert_allclose(cd, c1, rtol=1e-10, atol=1e-10)


def _count_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    from tensorflow_distributed_clustering_amd.parallel import dist as D
    D._COMM = None
    comm = D.init_comm("cpu")
    # synthetic per-rank cluster counts far above 2^24 (a 2^31-row shard's worth)
    c = torch.tensor([3 * 2 ** 24 + 12345 * rank + 7, 2 ** 31 - 1 - rank, 0, 1 + rank,
                      2 ** 24 + 1], dtype=torch.int64)
    hi = torch.zeros(5, dtype=torch.float32)
    lo = torch.zeros(5, dtype=torch.float32)
    D.split_counts(c, hi, lo)
    buf = torch.cat([hi, lo])
    comm.allreduce_bucketed_(buf, 8)  # 2-element buckets: also the bucketed branch
    naive = c.to(torch.float32)
    comm.allreduce_(naive)
    q.put((rank, D.join_counts(buf[:5], buf[5:]).numpy(), naive.double().numpy()))
    D.destroy_comm()


def test_counts_above_2p24_exact_through_fp32_allreduce():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_count_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (a, b)) for r, a, b in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exact = sum(np.array([3 * 2 ** 24 + 12345 * r + 7, 2 ** 31 - 1 - r, 0, 1 + r, 2 ** 24 + 1],
                         dtype=np.int64) for r in range(world))
    for r in range(world):
        np.testing.assert_array_equal(res[r][0], exact.astype(np.float64))
    assert not np.array_equal(res[0][1], exact.astype(np.float64))  # plain fp32 is not exact


def _split_worker(rank, world, port, policy, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.parallel import dist as D
    D._COMM = None
    comm = D.init_comm("cpu")
    # rank 0 owns only points near (0,0), rank 1 only points near (10,10)
    g = torch.Generator().manual_seed(rank)
    x = torch.randn(500, 2, generator=g, dtype=torch.float64) * 0.1 + 10.0 * rank
    cfg = tdc.ClusterConfig(n_clusters=2, max_iter=1, dtype="fp64", empty_cluster=policy)
    r = tdc.KMeans(cfg, comm).fit(x, init_centers_=np.array([[0.0, 0.0], [10.0, 10.0]]),
                                  n_global=1000, row_offset=500 * rank).result_
    if rank == 0:
        q.put(r.centers)
    D.destroy_comm()


def _run_split(policy):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_worker, args=(r, 2, port, policy, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return out


def test_nan_any_poisons_cluster_empty_on_one_rank():
    # each cluster is empty on one of the two ranks: the script's per-GPU reduce_mean
    # poisons both centroids ('nan_any'); the globally-empty rule ('nan') does not
    assert np.isnan(_run_split("nan_any")).all()
    c = _run_split("nan")
    assert not np.isnan(c).any()
    np.testing.assert_allclose(c, [[0, 0], [10, 10]], atol=0.05)


def _mismatch_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from tensorflow_distributed_clustering_amd.parallel import dist as D
    D._COMM = None
    comm = D.init_comm("cpu", timeout_s=60, debug=True)
    comm.allreduce_(torch.ones(4, dtype=torch.float64))  # consistent: passes
    err = ""
    try:  # rank 1 reduces a different shape (a diverged rank)
        comm.allreduce_(torch.ones(4 if rank == 0 else 5, dtype=torch.float64))
    except RuntimeError as e:
        err = str(e)
    q.put((rank, err))
    D.destroy_comm()


def test_dist_debug_detects_collective_mismatch():
    """--dist_debug (TORCH_DISTRIBUTED_DEBUG=DETAIL): a rank issuing a mismatched
    collective raises on every rank instead of hanging or reducing garbage."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mismatch_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    assert all(res[r] for r in (0, 1)), res
    assert any("shape" in res[r].lower() or "mismatch" in res[r].lower() for r in (0, 1)), res


def test_large_k_kmeanspp_is_sampled_kmeans_parallel_world_invariant(monkeypatch):
    """Above KPP_MAX_K, init='kmeans++' seeds with k-means|| on a world-invariant uniform
    sample (greedy k-means++ would be K dependent sweeps): same centres at world 1 and 2."""
    _, _, _, _, i1, _ = run_world(1, init="kmeans++", k=24, iters=1, extra=dict(kpp_max_k=8))
    _, _, _, _, i2, _ = run_world(2, init="kmeans++", k=24, iters=1, extra=dict(kpp_max_k=8))
    np.testing.assert_allclose(i2, i1, rtol=1e-12, atol=1e-12)
    assert len(np.unique(i1, axis=0)) == 24


def test_sampled_greedy_kmeanspp_world_invariant_and_sound():
    """N > 4 * max(min sample, kpp_sample_per_k * K): greedy k-means++ runs on a uniform
    world-invariant sample.  Same seeds at world 1 and 2, every seed is a data row, and the
    seeding is as good as greedy k-means++ over all rows (potential within 2x; the blobs are
    well separated, so both find one seed per blob)."""
    extra = dict(kpp_sample_per_k=200, kpp_sample_min=1000)
    n, k = 30011, 6
    c1, _, in1, _, i1, _ = run_world(1, init="kmeans++", n=n, k=k, iters=0, extra=extra)
    _, _, _, _, i2, _ = run_world(2, init="kmeans++", n=n, k=k, iters=0, extra=extra)
    np.testing.assert_allclose(i2, i1, rtol=1e-12, atol=1e-12)
    from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
    x = gaussian_blobs(n, 3, k, seed=11, dtype=torch.float64)
    d = torch.cdist(torch.as_tensor(i1), x).min(1).values
    assert float(d.max()) < 1e-9  # seeds are data rows
    _, _, _, _, full, _ = run_world(1, init="kmeans++", n=n, k=k, iters=0,
                                    extra=dict(kpp_sample_per_k=0))
    pot = lambda c: float(torch.cdist(x, torch.as_tensor(c)).min(1).values.pow(2).sum())
    assert pot(i1) < 2.0 * pot(full)


def _warmup_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.data.stream import PlainHostSource
    from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
    from tensorflow_distributed_clustering_amd.models.kmeans import LloydEngine
    from tensorflow_distributed_clustering_amd.parallel import dist as D
    D._COMM = None
    comm = D.init_comm("cpu")
    s, e = comm.shard(4000)
    x = gaussian_blobs(e - s, 3, 4, seed=1, row_offset=s, dtype=torch.float64)
    cfg = tdc.ClusterConfig(n_clusters=4, max_iter=3, dtype="fp64", seed=2, init="first_k")
    # rank 1 streams its shard (a planner may pick that for one rank only), rank 0 is resident
    src = PlainHostSource(x.numpy(), (torch.float64, 3), torch.device("cpu"), s) if rank else x
    eng = LloydEngine(src, cfg, comm, 4000, s, chunk_rows=500 if rank else 0)
    c0 = eng.C.clone()
    eng.warmup(force=True)  # collective decision: rank 1 cannot, so neither warms up
    same = bool(torch.equal(eng.C, c0)) and eng.n_iter == 0
    # the streamed rank cannot run the delta update, so no rank does (one buffer layout,
    # one mode per step)
    same = same and eng.update_mode == "full"
    for _ in range(2):
        eng.step()
    q.put((rank, same, eng.C.numpy().copy()))
    D.destroy_comm()


def test_warmup_is_skipped_on_every_rank_when_one_rank_streams():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_warmup_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (a, b)) for r, a, b in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] and res[1][0]
    np.testing.assert_array_equal(res[0][1], res[1][1])


def test_forced_collectives_world1_equals_local(monkeypatch):
    """TDC_FORCE_COLLECTIVES=1: a world-1 process group that issues every collective (the
    single-GPU RCCL rehearsal of tests/test_rccl_gpu.py) gives the no-group result; rsag
    engages at world 1 only when forced."""
    c0, l0, in0, it0, i0, f0 = run_world(1, extra={"comm_mode": "rsag"})
    monkeypatch.setenv("TDC_FORCE_COLLECTIVES", "1")
    c1, l1, in1, it1, i1, f1 = run_world(1)
    np.testing.assert_array_equal(c1, c0)
    np.testing.assert_array_equal(l1, l0)
    assert it1 == it0
    c2, l2, _, _, _, f2 = run_world(1, extra={"comm_mode": "rsag"})
    assert f2["rsag"] and not f0["rsag"]
    np.testing.assert_allclose(c2, c0, rtol=1e-12, atol=1e-12)
    np.testing.assert_array_equal(l2, l0)
