"""Multi-rank GPU path on ONE MI355X: ranks share cuda:0 and talk over gloo
(``TDC_DIST_BACKEND=gloo``; RCCL refuses two ranks on one device).  Everything but the
transport is the production path: on-device shard generation, world-size-invariant
init, the HIP kernels, the packed all-reduce of [sums | counts] and the replicated
finalize.  World 2 must reproduce world 1 (up to float-atomic summation order).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q, dtype, n, d, k, iters, method, algorithm="lloyd",
            comm_mode="auto", extra=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank), TDC_DIST_BACKEND="gloo")
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
    from tensorflow_distributed_clustering_amd.parallel import dist as D
    D._COMM = None
    comm = D.init_comm("cuda")
    s, e = comm.shard(n)
    tdt = {"bf16": torch.bfloat16, "fp8": torch.bfloat16, "fp32": torch.float32,
           "fp64": torch.float64}[dtype]
    x = gaussian_blobs(e - s, d, k, seed=3, row_offset=s, dtype=tdt, device=comm.device)
    cfg = tdc.ClusterConfig(n_clusters=k, max_iter=iters, dtype=dtype, init="random", seed=3,
                            algorithm=algorithm, comm_mode=comm_mode, **(extra or {}))
    model = (tdc.KMeans if method == "kmeans" else tdc.FuzzyCMeans)(cfg, comm)
    model.fit(x, n_global=n, row_offset=s)
    r = model.result_
    labels = comm.gather_rows_to_root(torch.as_tensor(r.labels, device=comm.device))
    eng = model.engine_
    info = dict(rsag=getattr(eng, "rsag", False), split=getattr(eng, "count_split", False),
                counts=r.counts, update_mode=getattr(eng, "update_mode", None),
                update_stats=eng.update_stats() if hasattr(eng, "update_stats") else None)
    if rank == 0:
        q.put((np.asarray(r.centers), labels.cpu().numpy(), r.backend, info))
    D.destroy_comm()


def _run(world, dtype, n, d, k, iters=4, method="kmeans", algorithm="lloyd", comm_mode="auto",
         full=False, extra=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker,
                         args=(r, world, port, q, dtype, n, d, k, iters, method, algorithm,
                               comm_mode, extra))
             for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out if full else out[:3]


@pytest.mark.parametrize("world,dtype,d,k", [(2, "bf16", 128, 1000), (3, "bf16", 128, 1000),
                                             (2, "fp8", 256, 500), (2, "fp32", 96, 700),
                                             # K=40 over 3 ranks of 32-row slices: rank 2's
                                             # slice has no real centroid (fp8 finalize of
                                             # an empty slice, padding rows only)
                                             (3, "fp8", 256, 40)])
def test_rsag_matches_one_rank(gpu, world, dtype, d, k):
    """comm_mode='rsag': reduce-scatter of the fp32 sums, each rank finalises + preps the
    operand rows of its K/G slice, all-gather of the bf16/fp8 operand tables (fp32 path:
    the centroids); K is not a multiple of 64 x G, so the padded tail slice is covered.
    The fp32 buffers also carry the exact count halves."""
    n = 120_001
    c1, l1, b1, i1 = _run(1, dtype, n, d, k, full=True)
    c2, l2, b2, i2 = _run(world, dtype, n, d, k, comm_mode="rsag", full=True)
    assert b1 == b2 and i2["rsag"] and not i1["rsag"]
    if k * (d + 1) > 65536:  # fp32 partial sums (smaller buffers travel in fp64)
        assert i1["split"] and i2["split"]
    assert i2["counts"].sum() == n and np.all(i2["counts"] == np.round(i2["counts"]))
    if dtype == "fp32":
        np.testing.assert_allclose(c2, c1, rtol=1e-4, atol=1e-4)
    else:
        # bf16/fp8 distances: a last-bit difference of the reduced sums can flip a near-tie
        # assignment, moving a centroid or two by a fraction of a point; the rest agree
        ok = np.isclose(c2, c1, rtol=2e-3, atol=2e-3).all(1)
        assert ok.mean() > 0.99, ok.mean()
    assert (l1 == l2).mean() > 0.99


def test_bf16_mfma_two_ranks_match_one(gpu):
    c1, l1, b1 = _run(1, "bf16", 200_003, 128, 256)
    c2, l2, b2 = _run(2, "bf16", 200_003, 128, 256)
    assert b1 == b2 == "hip_bf16_mfma"
    np.testing.assert_allclose(c2, c1, rtol=1e-3, atol=1e-3)
    assert (l1 == l2).mean() > 0.999


def test_fp64_fused_two_ranks_match_one(gpu):
    c1, l1, _ = _run(1, "fp64", 100_001, 5, 3)
    c2, l2, _ = _run(2, "fp64", 100_001, 5, 3)
    np.testing.assert_allclose(c2, c1, rtol=1e-10, atol=1e-10)
    np.testing.assert_array_equal(l2, l1)


def test_fcm_two_ranks_match_one(gpu):
    c1, l1, _ = _run(1, "fp64", 50_000, 5, 4, method="fcm")
    c2, l2, _ = _run(2, "fp64", 50_000, 5, 4, method="fcm")
    np.testing.assert_allclose(c2, c1, rtol=1e-9, atol=1e-9)
    np.testing.assert_array_equal(l2, l1)


@pytest.mark.parametrize("dtype,d,k", [("fp64", 128, 256), ("fp32", 64, 128)])
def test_fcm_f64_mfma_two_ranks_match_one(gpu, dtype, d, k):
    """FCM on the fp64 matrix-core path (fused row statistics; fp32 rows promoted) at
    world 2: each rank's partial W^T X / sum W through the packed all-reduce reproduces the
    one-rank fit."""
    c1, l1, b1 = _run(1, dtype, 40_001, d, k, iters=3, method="fcm", extra={"fuzzifier": 2.0})
    c2, l2, b2 = _run(2, dtype, 40_001, d, k, iters=3, method="fcm", extra={"fuzzifier": 2.0})
    assert b1 == b2 == "hip_fcm_wide"
    np.testing.assert_allclose(c2, c1, rtol=1e-9, atol=1e-9)
    assert (l1 == l2).mean() > 0.9999


def test_bounded_two_ranks_match_lloyd(gpu):
    """algorithm='bounded' on 2 ranks: per-rank pruning, one all-reduce of the deltas per
    step, replicated fp64 totals -> the single-rank Lloyd result."""
    c1, l1, _ = _run(1, "bf16", 200_003, 128, 1024, iters=12)
    c2, l2, b2 = _run(2, "bf16", 200_003, 128, 1024, iters=12, algorithm="bounded")
    assert b2 == "hip_bf16_mfma"
    np.testing.assert_allclose(c2, c1, rtol=2e-3, atol=2e-3)
    assert (l1 == l2).mean() > 0.999


@pytest.mark.parametrize("world,dtype,d,k,comm_mode", [
    (2, "bf16", 128, 1000, "allreduce"), (3, "bf16", 128, 1000, "allreduce"),
    (2, "bf16", 128, 1000, "rsag"), (2, "fp8", 256, 500, "rsag"),
    (3, "fp8", 256, 40, "rsag"),  # rank 2's slice: padding rows only
    (2, "fp32", 96, 700, "rsag")])
@pytest.mark.parametrize("mode", ["refresh2", "theta0"])
def test_native_delta_multi_rank(gpu, world, dtype, d, k, comm_mode, mode):
    """The native delta update across ranks (HIP diff / scan / scatter / segsum kernels,
    device-side full/delta choice from the all-reduced moved count): with a refresh every
    2 steps, or theta = 0 (any moved row makes the next step full), the ranks switch
    modes together (the run completes and the stats count full steps) and the fit matches
    update='full' at the same world size -- also under reduce-scatter mode, where each rank
    keeps only its slice of the fp64 totals."""
    n, iters = 120_001, 7
    extra = ({"delta_refresh": 2} if mode == "refresh2" else
             {"delta_refresh": 0, "delta_theta": 0.0})
    cf, lf, bf, fi = _run(world, dtype, n, d, k, iters, comm_mode=comm_mode, full=True,
                          extra={"update": "full"})
    cd, ld, bd, di = _run(world, dtype, n, d, k, iters, comm_mode=comm_mode, full=True,
                          extra=dict(update="delta", **extra))
    assert bf == bd and di["update_mode"] == "delta" and fi["update_mode"] == "full"
    assert di["rsag"] == (comm_mode == "rsag")
    st = di["update_stats"]
    assert st["full_steps"] >= 2 and st["full_steps"] < st["steps"], st
    if mode == "theta0":
        assert st["moved_rows"] > 0
    assert di["counts"].sum() == n
    if dtype == "fp32":
        np.testing.assert_allclose(cd, cf, rtol=1e-4, atol=1e-4)
    else:
        ok = np.isclose(cd, cf, rtol=2e-3, atol=2e-3).all(1)
        assert ok.mean() > 0.99, ok.mean()
    assert (lf == ld).mean() > 0.99
