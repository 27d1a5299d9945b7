"""Every RCCL call of the production path on ONE MI355X.

RCCL refuses two ranks on one device, and at world size 1 the communicator short-circuits
its collectives, so the multi-rank tests (tests/test_dist_gpu.py) run over gloo.  Here a
world-1 RCCL ("nccl") process group is created with ``TDC_FORCE_COLLECTIVES=1``: the
packed all-reduce (one call and bucketed), reduce-scatter + all-gather (bf16 and fp8
operand tables), the int64/fp64 scalar reductions of the init and the OOM/warm-up
agreement, barriers and the label gather all go through RCCL.  A sum over one rank is
that rank's value, so the fits must equal the same fits on a communicator without a
process group (up to float-atomic summation order; rsag: up to its sliced finalize).
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


CASES = [
    # name, dtype, n, d, k, iters, method, extra cfg
    ("allreduce", "bf16", 200_003, 128, 256, 4, "kmeans", {}),
    ("bucketed", "bf16", 200_003, 128, 256, 4, "kmeans", {"bucket_kb": 48}),
    ("rsag", "bf16", 120_001, 128, 1000, 4, "kmeans", {"comm_mode": "rsag"}),
    ("rsag_fp8", "fp8", 60_001, 256, 500, 3, "kmeans", {"comm_mode": "rsag"}),
    ("fused_fp64", "fp64", 100_001, 5, 3, 5, "kmeans", {}),
    ("fcm_fp64", "fp64", 50_000, 5, 4, 5, "fcm", {}),
    ("bounded", "bf16", 200_003, 128, 1024, 12, "kmeans", {"algorithm": "bounded"}),
    ("deterministic", "bf16", 200_003, 128, 256, 5, "kmeans", {"deterministic": True}),
]


def _worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="1",
                      RANK="0", LOCAL_RANK="0", TDC_FORCE_COLLECTIVES="1")
    os.environ.pop("TDC_DIST_BACKEND", None)
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
    from tensorflow_distributed_clustering_amd.parallel import dist as D
    D._COMM = None
    comm = D.init_comm("cuda")
    local = D.local_comm(comm.device)
    out = {"backend": comm.backend, "collective": comm.collective,
           "local_collective": local.collective}
    for name, dtype, n, d, k, iters, method, extra in CASES:
        tdt = {"bf16": torch.bfloat16, "fp8": torch.bfloat16, "fp64": torch.float64}[dtype]
        x = gaussian_blobs(n, d, k, seed=5, dtype=tdt, device=comm.device)
        res = []
        for cm in (comm, local):
            cfg = tdc.ClusterConfig(n_clusters=k, max_iter=iters, dtype=dtype, init="random",
                                    seed=5, **extra)
            model = (tdc.KMeans if method == "kmeans" else tdc.FuzzyCMeans)(cfg, cm)
            model.fit(x, n_global=n, row_offset=0)
            r = model.result_
            labels = cm.gather_rows_to_root(torch.as_tensor(r.labels, device=cm.device))
            res.append((np.asarray(r.centers), labels.cpu().numpy(),
                        bool(getattr(model.engine_, "rsag", False))))
        out[name] = res
    # the whole step captured into a hipGraph WITH its RCCL all-reduce (the multi-GPU
    # bench's --graph path) against eager steps on the same group; delta update on
    from tensorflow_distributed_clustering_amd.models.kmeans import LloydEngine
    n, d, k = 200_003, 128, 256
    x = gaussian_blobs(n, d, k, seed=7, dtype=torch.bfloat16, device=comm.device)
    cfg = tdc.ClusterConfig(n_clusters=k, max_iter=8, dtype="bf16", init="random", seed=7,
                            delta_refresh=3)
    res = []
    for graph in (False, True):
        eng = LloydEngine(x, cfg, comm, n, 0)
        if graph:
            eng.capture(include_collectives=True)
        for _ in range(8):
            eng.step()
        torch.cuda.synchronize()
        res.append((eng.C.cpu().numpy(), eng.update_mode, eng._graph is not None
                    if hasattr(eng, "_graph") else False))
    out["graph"] = res
    comm.barrier()
    q.put(out)
    D.destroy_comm()


@pytest.fixture(scope="module")
def rccl_results(gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    out = q.get(timeout=110)
    p.join(timeout=60)
    assert p.exitcode == 0
    return out


def test_rccl_process_group(rccl_results):
    assert rccl_results["backend"] == "nccl"  # RCCL on ROCm
    assert rccl_results["collective"] and not rccl_results["local_collective"]


@pytest.mark.parametrize("name", ["allreduce", "bucketed", "fused_fp64", "fcm_fp64"])
def test_rccl_allreduce_paths_equal_local(rccl_results, name):
    """Equal up to the float-atomic summation order of the update kernels (two local runs
    differ in the last bit too)."""
    (c_r, l_r, _), (c_l, l_l, _) = rccl_results[name]
    if name.endswith("fp64"):
        np.testing.assert_allclose(c_r, c_l, rtol=1e-10, atol=1e-10)
        np.testing.assert_array_equal(l_r, l_l)
    else:
        np.testing.assert_allclose(c_r, c_l, rtol=1e-5, atol=1e-5)
        assert (l_r == l_l).mean() > 0.999


@pytest.mark.parametrize("name", ["rsag", "rsag_fp8"])
def test_rccl_rsag_matches_local(rccl_results, name):
    (c_r, l_r, rsag_r), (c_l, l_l, rsag_l) = rccl_results[name]
    assert rsag_r and not rsag_l
    ok = np.isclose(c_r, c_l, rtol=2e-3, atol=2e-3).all(1)
    assert ok.mean() > 0.99, ok.mean()
    assert (l_r == l_l).mean() > 0.99


def test_rccl_bounded_matches_local(rccl_results):
    (c_r, l_r, _), (c_l, l_l, _) = rccl_results["bounded"]
    np.testing.assert_allclose(c_r, c_l, rtol=2e-3, atol=2e-3)
    assert (l_r == l_l).mean() > 0.999


def test_rccl_graph_capture_with_collectives_equals_eager(rccl_results):
    """capture(include_collectives=True) on the RCCL group: replayed steps (all-reduce
    inside the graph) reach the eager steps' centroids."""
    (c_e, mode_e, g_e), (c_g, mode_g, g_g) = rccl_results["graph"]
    assert not g_e and g_g and mode_e == mode_g == "delta"
    np.testing.assert_allclose(c_g, c_e, rtol=1e-5, atol=1e-5)


def test_rccl_deterministic_int64_allreduce_bitwise(rccl_results):
    """Fixed-point partials through an int64 RCCL all-reduce: the RCCL fit equals the
    no-group fit bit for bit (integer sums do not depend on any reduction order)."""
    (c_r, l_r, _), (c_l, l_l, _) = rccl_results["deterministic"]
    assert np.array_equal(c_r, c_l)
    np.testing.assert_array_equal(l_r, l_l)
