"""GPU: streamed Lloyd (host pinned ring + copy stream, on-device generator) and mini-batch
K-Means through the HIP kernels, checked against the resident HIP run and fp64 truth."""
import numpy as np
import pytest
import torch

import tensorflow_distributed_clustering_amd as tdc
from tensorflow_distributed_clustering_amd.data.stream import HostSource, SyntheticSource
from tensorflow_distributed_clustering_amd.data.synth import blob_centers, gaussian_blobs

pytestmark = pytest.mark.gpu


def test_host_source_h2d_ring(gpu):
    x = np.random.default_rng(1).normal(size=(70001, 100)).astype(np.float32)
    hs = HostSource(x, (torch.bfloat16, 128), gpu, n_pinned=3, n_threads=4)
    parts = [c.clone() for _, c in hs.chunks(9000)]
    got = torch.cat(parts).cpu()
    ref = torch.zeros(70001, 128, dtype=torch.bfloat16)
    ref[:, :100] = torch.from_numpy(x).to(torch.bfloat16)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_host_streamed_lloyd_matches_resident(gpu, dtype):
    xh = gaussian_blobs(200_000, 32, 16, seed=3, dtype=torch.float32).numpy()
    cfg = tdc.ClusterConfig(n_clusters=16, max_iter=6, dtype=dtype, seed=5)
    a = tdc.KMeans(cfg, device=gpu).fit(torch.from_numpy(xh).to(gpu))
    b = tdc.KMeans(cfg.replace(chunk_rows=30_000), device=gpu).fit(xh)
    assert b.result_.streamed and not a.result_.streamed
    assert b.result_.backend == a.result_.backend
    np.testing.assert_allclose(b.result_.centers, a.result_.centers, rtol=1e-4, atol=1e-4)
    agree = (a.result_.labels == b.result_.labels).float().mean().item()
    assert agree > 0.999
    assert abs(b.result_.inertia - a.result_.inertia) <= 1e-4 * a.result_.inertia


def test_synthetic_source_bf16_stream(gpu):
    n, d, k = 300_000, 64, 32
    src = SyntheticSource(n, d, k, seed=9, row_offset=0, layout=(torch.bfloat16, 64), device=gpu)
    cfg = tdc.ClusterConfig(n_clusters=k, max_iter=10, dtype="bf16", seed=1, init="kmeans++",
                            chunk_rows=65536)
    km = tdc.KMeans(cfg, device=gpu).fit(src, n_global=n, row_offset=0)
    assert km.result_.streamed and km.result_.backend == "hip_bf16_mfma"
    true_c = blob_centers(k, d, 9)
    dist = ((km.result_.centers[:, None] - true_c[None]) ** 2).sum(-1)
    assert np.median(dist.min(1)) < 1.0


def test_minibatch_gpu_bf16(gpu):
    n, d, k = 400_000, 64, 64
    x = gaussian_blobs(n, d, k, seed=4, dtype=torch.bfloat16, device=gpu)
    cfg = tdc.ClusterConfig(n_clusters=k, max_iter=60, dtype="bf16", seed=3, init="kmeans++",
                            batch_size=32768)
    mb = tdc.MiniBatchKMeans(cfg, device=gpu).fit(x)
    full = tdc.KMeans(tdc.ClusterConfig(n_clusters=k, max_iter=20, dtype="bf16", seed=3,
                                        init="kmeans++"), device=gpu).fit(x)
    assert mb.result_.backend == "hip_bf16_mfma"
    assert mb.result_.inertia <= 1.10 * full.result_.inertia


def test_minibatch_gpu_indexed_path(gpu):
    """K x D past the LDS update: the mini-batch step samples row indices and the kernels
    read the rows in place (+ the native Sculley update); quality vs full-batch Lloyd."""
    n, d, k = 600_000, 128, 1024
    x = gaussian_blobs(n, d, 256, seed=6, dtype=torch.bfloat16, device=gpu)
    cfg = tdc.ClusterConfig(n_clusters=k, max_iter=40, dtype="bf16", seed=3, batch_size=65536)
    mb = tdc.MiniBatchKMeans(cfg, device=gpu).fit(x)
    assert mb.engine_._indexed() and mb.result_.backend == "hip_bf16_mfma"
    assert int(mb.result_.counts.sum()) == 40 * 65536
    full = tdc.KMeans(tdc.ClusterConfig(n_clusters=k, max_iter=10, dtype="bf16", seed=3),
                      device=gpu).fit(x)
    assert mb.result_.inertia <= 1.15 * full.result_.inertia


@pytest.mark.parametrize("dtype,d,k", [("bf16", 128, 256), ("fp64", 5, 3), ("fp8", 256, 96)])
def test_graph_replay_matches_eager(gpu, dtype, d, k):
    x = gaussian_blobs(100_000, d, k, seed=2, dtype=torch.float32, device=gpu)
    cfg = tdc.ClusterConfig(n_clusters=k, max_iter=7, dtype=dtype, seed=4)
    eager = tdc.KMeans(cfg, device=gpu).fit(x).result_
    graph = tdc.KMeans(cfg.replace(graph=True), device=gpu).fit(x).result_
    assert graph.n_iter == eager.n_iter == 7
    if dtype == "fp8":
        # float atomics in the update differ in the last bits between two runs (graph or
        # not); re-quantising the centroids to fp8 can turn that into a flipped near-tie
        # row, which moves its two centroids by ~|x - c| / count: compare per centroid
        ok = np.isclose(graph.centers, eager.centers, rtol=1e-5, atol=1e-5).all(1)
        assert ok.mean() >= 0.97, ok.mean()
    else:
        np.testing.assert_allclose(graph.centers, eager.centers, rtol=1e-5, atol=1e-5)
    assert (graph.labels == eager.labels).float().mean().item() > 0.999


def test_deterministic_mode_bitwise_reproducible(gpu):
    x = gaussian_blobs(300_000, 64, 512, seed=8, dtype=torch.bfloat16, device=gpu)
    cfg = tdc.ClusterConfig(n_clusters=512, max_iter=5, dtype="bf16", seed=1, deterministic=True)
    a = tdc.KMeans(cfg, device=gpu).fit(x).result_
    b = tdc.KMeans(cfg, device=gpu).fit(x).result_
    assert np.array_equal(a.centers, b.centers)
    assert torch.equal(a.labels, b.labels)


def test_per_iteration_inertia_on_gpu(gpu):
    x = gaussian_blobs(200_000, 32, 64, seed=3, dtype=torch.bfloat16, device=gpu)
    r = tdc.KMeans(tdc.ClusterConfig(n_clusters=64, max_iter=6, dtype="bf16", log_every=1,
                                     seed=2), device=gpu).fit(x).result_
    inert = [h["inertia"] for h in r.history]
    assert len(inert) == 6 and all(b <= a * 1.0001 for a, b in zip(inert, inert[1:]))


def test_hybrid_resident_host_stream(gpu):
    xh = gaussian_blobs(150_000, 32, 16, seed=3, dtype=torch.float32).numpy()
    hs = HostSource(xh, (torch.bfloat16, 32), gpu, resident_rows=70_000)
    for _ in range(2):  # second pass reuses the resident prefix
        got = torch.cat([c.clone() for _, c in hs.chunks(25_000)]).cpu()
        assert torch.equal(got, torch.from_numpy(xh).to(torch.bfloat16))
    cfg = tdc.ClusterConfig(n_clusters=16, max_iter=5, dtype="bf16", seed=5, hbm_budget_gb=0.02)
    a = tdc.KMeans(cfg, device=gpu).fit(xh)  # tiny budget -> planner streams + keeps a prefix
    b = tdc.KMeans(cfg.replace(hbm_budget_gb=0.0), device=gpu).fit(torch.from_numpy(xh).to(gpu))
    assert a.result_.streamed
    np.testing.assert_allclose(a.result_.centers, b.result_.centers, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_spherical_kmeans_gpu_bf16(gpu):
    g = torch.Generator().manual_seed(3)
    dirs = torch.nn.functional.normalize(torch.randn(32, 128, generator=g), dim=1)
    lab = torch.randint(0, 32, (200_000,), generator=g)
    x = (dirs[lab] + 0.02 * torch.randn(200_000, 128, generator=g)) * (1 + 5 * torch.rand(200_000, 1, generator=g))
    r = tdc.KMeans(tdc.ClusterConfig(n_clusters=32, max_iter=10, dtype="bf16", spherical=True,
                                     init="kmeans++", seed=0)).fit(x.cuda()).result_
    c = torch.as_tensor(r.centers).float().cpu()
    torch.testing.assert_close(c.norm(dim=1), torch.ones(32), atol=1e-2, rtol=0)
    assert (dirs @ c.t()).max(1).values.min() > 0.98


@pytest.mark.parametrize("d,k,policy", [(128, 1024, "keep"), (64, 4096, "keep"), (256, 300, "zero")])
def test_bounded_lloyd_matches_lloyd(gpu, d, k, policy):
    """algorithm='bounded' (Hamerly bounds: re-assign only unsettled rows, incremental
    totals) reaches Lloyd's result and prunes most rows once the centroids settle."""
    x = gaussian_blobs(300_000, d, k, seed=11, dtype=torch.bfloat16, device=gpu)
    cfg = tdc.ClusterConfig(n_clusters=k, max_iter=25, dtype="bf16", seed=5, init="kmeans++",
                            empty_cluster=policy)
    a = tdc.KMeans(cfg, device=gpu).fit(x)
    b = tdc.KMeans(cfg.replace(algorithm="bounded"), device=gpu).fit(x)
    assert b.engine_.enabled and type(b.engine_).__name__ == "BoundedLloydEngine"
    assert abs(a.result_.inertia - b.result_.inertia) <= 1e-4 * a.result_.inertia
    agree = (a.result_.labels == b.result_.labels).float().mean().item()
    assert agree > 0.999
    assert b.engine_.active_frac < 0.9  # data dependent; 8-12 % on the headline config
    np.testing.assert_allclose(b.result_.counts.sum(), 300_000)


def test_bounded_lloyd_policies_and_spherical(gpu):
    """bounded == Lloyd also with NaN-poisoned empty clusters (a centroid that turns NaN
    re-assigns every row once, then drops out of the drift), with empty clusters re-seeded
    (reseed must read the totals, not the step's deltas) and for spherical K-Means
    (centroids re-normalised after each update)."""
    x = gaussian_blobs(200_000, 128, 300, seed=3, dtype=torch.bfloat16, device=gpu)
    base = tdc.ClusterConfig(n_clusters=512, max_iter=12, dtype="bf16", seed=2, init="random")
    for cfg in (base.replace(empty_cluster="nan"), base.replace(empty_cluster="reseed"),
                base.replace(spherical=True)):
        a = tdc.KMeans(cfg, device=gpu).fit(x).result_
        bm = tdc.KMeans(cfg.replace(algorithm="bounded"), device=gpu).fit(x)
        b = bm.result_
        agree = (a.labels == b.labels).float().mean().item()
        assert agree > 0.999, (cfg.empty_cluster, cfg.spherical, agree)
        np.testing.assert_array_equal(np.isnan(a.centers).any(1), np.isnan(b.centers).any(1))
        if cfg.empty_cluster == "nan":
            assert np.isnan(b.centers).any()       # the case under test happened
            assert bm.engine_.active_frac < 0.9    # NaN centroids no longer force full passes
        if cfg.empty_cluster == "reseed":
            np.testing.assert_allclose(a.centers, b.centers, rtol=0, atol=5e-2)


@pytest.mark.parametrize("dtype,backend", [("bf16", "hip_fcm_mfma"), ("fp32", "hip_fcm_wide"),
                                           ("fp64", "hip_fcm_wide")])
def test_fcm_hbm_budget_streams_and_matches_resident(gpu, dtype, backend):
    """FCM with --hbm_budget_gb below the shard: host-resident rows stream through HBM in
    chunks (fp32: native RowStreamer + hybrid residency; fp64: plain pinned slices) and
    the result equals the resident fit (same partials, summed over chunks)."""
    import numpy as np
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
    n, d, k = 400_000, 64, 64  # fp32 / fp64: the fused fp64 MFMA path (fp32 chunks widened)
    x = gaussian_blobs(n, d, k, seed=6, dtype=torch.float64).numpy()
    c0 = x[:k] + 0.3
    cfg = tdc.ClusterConfig(n_clusters=k, max_iter=4, dtype=dtype, init="given", fuzzifier=2.0)
    res = tdc.FuzzyCMeans(cfg, device=gpu).fit(x, init_centers_=c0).result_
    st = tdc.FuzzyCMeans(cfg.replace(hbm_budget_gb=0.05), device=gpu).fit(x, init_centers_=c0).result_
    assert not res.streamed and st.streamed and res.backend == st.backend == backend
    tol = 1e-9 if dtype == "fp64" else 2e-4
    np.testing.assert_allclose(st.centers, res.centers, rtol=tol, atol=tol)
    assert (st.labels == res.labels).float().mean().item() > 0.999


def _fp64_shard(n=2_000_000, d=16, k=16):
    x = gaussian_blobs(n, d, k, seed=12, dtype=torch.float64).numpy()
    return x, x[:k] + 0.25


def test_fp64_kmeans_larger_than_budget_streams_from_host(gpu):
    """fp64 K-Means (the reference's dtype) with an HBM budget below the shard: the rows
    stay in host memory and stream through the RowStreamer's pinned ring (f64 rows as they
    are) into the fused fp64 kernel; same centres as the resident fit to 1e-9, and the
    device never holds the shard (peak allocation well below the shard's bytes)."""
    x, c0 = _fp64_shard()
    cfg = tdc.ClusterConfig(n_clusters=16, max_iter=5, dtype="fp64", init="given")
    res = tdc.KMeans(cfg, device=gpu).fit(x, init_centers_=c0).result_
    del_labels = res.labels
    res.labels = None
    del del_labels
    torch.cuda.synchronize(gpu)
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(gpu)
    base = torch.cuda.memory_allocated(gpu)
    st = tdc.KMeans(cfg.replace(hbm_budget_gb=0.1), device=gpu).fit(x, init_centers_=c0).result_
    peak = torch.cuda.max_memory_allocated(gpu) - base
    assert st.streamed and not res.streamed and st.backend == res.backend
    np.testing.assert_allclose(st.centers, res.centers, rtol=1e-9, atol=1e-9)
    assert peak < 0.7 * x.nbytes, (peak, x.nbytes)


@pytest.mark.parametrize("fault", ["oom@setup", "oom@3"])
def test_fp64_kmeans_oom_falls_back_to_host_streaming(gpu, monkeypatch, fault):
    """TDC_FAULT=oom@setup (the upload of the fp64 shard fails) and oom@3 (iteration 3
    fails): the run continues streamed from host memory and matches the undisturbed fit;
    afterwards the device holds no copy of the shard (the failed engine was released)."""
    from tensorflow_distributed_clustering_amd.utils import faults
    x, c0 = _fp64_shard()
    cfg = tdc.ClusterConfig(n_clusters=16, max_iter=5, dtype="fp64", init="given")
    ref_c = tdc.KMeans(cfg, device=gpu).fit(x, init_centers_=c0).result_.centers
    torch.cuda.synchronize(gpu)
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(gpu)
    base = torch.cuda.memory_allocated(gpu)
    faults._FIRED.clear()
    monkeypatch.setenv("TDC_FAULT", fault)
    m = tdc.KMeans(cfg, device=gpu)
    r = m.fit(x, init_centers_=c0).result_
    monkeypatch.delenv("TDC_FAULT")
    faults._FIRED.clear()
    assert r.streamed
    np.testing.assert_allclose(r.centers, ref_c, rtol=1e-9, atol=1e-9)
    torch.cuda.synchronize(gpu)
    # the retry streams quarter-shard chunks through two device slots (half the shard)
    # next to the per-row labels / min distances (12 of the 128 bytes per row)
    now = torch.cuda.memory_allocated(gpu) - base
    assert now < 0.7 * x.nbytes, (now, x.nbytes)
    if fault == "oom@setup":
        assert torch.cuda.max_memory_allocated(gpu) - base < 0.7 * x.nbytes
    else:
        assert all(w() is None for w in m._retired)
