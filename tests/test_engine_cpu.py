"""Engine-level behaviour on CPU (torch backend): Lloyd == sklearn Lloyd, FCM, init,
empty-cluster handling, tolerance stop, label pass semantics."""
import numpy as np
import pytest
import torch

import tensorflow_distributed_clustering_amd as tdc
from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
from tensorflow_distributed_clustering_amd.models.init import floyd_sample
from tensorflow_distributed_clustering_amd.ops import reference as ref


def test_kmeans_matches_sklearn_lloyd():
    from sklearn.cluster import KMeans as SK
    x = gaussian_blobs(10000, 2, 8, seed=3)  # BASELINE config 1: 2-D blobs, N=10k, K=8
    km = tdc.KMeans(tdc.ClusterConfig(n_clusters=8, max_iter=20, dtype="fp64", seed=1)).fit(x)
    r = km.result_
    sk = SK(8, init=r.init_centers, n_init=1, max_iter=20, algorithm="lloyd", tol=0).fit(x.double().numpy())
    np.testing.assert_allclose(r.centers, sk.cluster_centers_, rtol=1e-9, atol=1e-9)
    assert abs(r.inertia - sk.inertia_) / sk.inertia_ < 1e-9
    assert r.n_iter == 20 and r.backend == "torch"
    np.testing.assert_array_equal(r.labels.numpy(), sk.labels_)


def test_label_pass_is_against_final_centers():
    x = gaussian_blobs(2000, 3, 4, seed=5, dtype=torch.float64)
    km = tdc.KMeans(tdc.ClusterConfig(n_clusters=4, max_iter=3, dtype="fp64")).fit(x)
    lab, _ = ref.assign(x, torch.as_tensor(km.result_.centers), exact=True)
    assert torch.equal(km.result_.labels, lab)


def test_tolerance_stops_early():
    x = gaussian_blobs(5000, 2, 3, seed=0, dtype=torch.float64)
    km = tdc.KMeans(tdc.ClusterConfig(n_clusters=3, max_iter=100, tol=1e-12, dtype="fp64")).fit(x)
    assert km.result_.n_iter < 100
    assert km.result_.history[-1]["shift"] <= 1e-12


def test_zero_iterations_returns_init():
    x = gaussian_blobs(100, 2, 3, seed=0, dtype=torch.float64)
    km = tdc.KMeans(tdc.ClusterConfig(n_clusters=3, max_iter=0, dtype="fp64", init="first_k")).fit(x)
    np.testing.assert_array_equal(km.result_.centers, x[:3].numpy())


@pytest.mark.parametrize("policy", ["keep", "nan", "zero", "reseed"])
def test_empty_cluster_policy_engine(policy):
    x = torch.cat([torch.zeros(50, 2), torch.ones(50, 2)]).double()
    init = np.array([[0.0, 0.0], [1.0, 1.0], [100.0, 100.0]])  # 3rd centroid gets no points
    km = tdc.KMeans(tdc.ClusterConfig(n_clusters=3, max_iter=2, dtype="fp64",
                                      empty_cluster=policy)).fit(x, init_centers_=init)
    c = km.result_.centers
    np.testing.assert_allclose(c[:2], [[0, 0], [1, 1]])
    if policy == "keep":
        np.testing.assert_allclose(c[2], [100, 100])
    elif policy == "nan":
        assert np.isnan(c[2]).all()
    elif policy == "zero":
        np.testing.assert_allclose(c[2], [0, 0])
    else:  # reseeded onto a data row
        assert ((c[2] == 0).all() or (c[2] == 1).all())


@pytest.mark.parametrize("init", ["random", "first_k", "kmeans++"])
def test_init_methods(init):
    x = gaussian_blobs(3000, 4, 6, seed=2, dtype=torch.float64)
    km = tdc.KMeans(tdc.ClusterConfig(n_clusters=6, max_iter=5, dtype="fp64", init=init, seed=4)).fit(x)
    c0 = km.result_.init_centers
    # every init center is a data row
    d = ((x.numpy()[:, None] - c0[None]) ** 2).sum(-1).min(0)
    assert np.all(d == 0)
    assert len({tuple(r) for r in c0}) == 6
    if init == "first_k":
        np.testing.assert_array_equal(c0, x[:6].numpy())


def test_floyd_sample_distinct_and_deterministic():
    a = floyd_sample(10 ** 9, 1000, 7)
    assert len(set(a)) == 1000 and all(0 <= v < 10 ** 9 for v in a)
    assert a == floyd_sample(10 ** 9, 1000, 7)
    assert sorted(floyd_sample(10, 10, 1)) == list(range(10))


def test_fcm_engine_matches_reference_iteration():
    x = gaussian_blobs(3000, 5, 3, seed=1, dtype=torch.float64)
    cfg = tdc.ClusterConfig(n_clusters=3, max_iter=4, dtype="fp64", init="first_k")
    f = tdc.FuzzyCMeans(cfg).fit(x)
    # oracle: m := D (compat), 4 iterations from X[0:3]
    c = x[:3].clone()
    for _ in range(4):
        wx, ws, _ = ref.fcm_partial(x, c, 5.0)
        c = wx / ws[:, None]
    np.testing.assert_allclose(f.result_.centers, c.numpy(), rtol=1e-10)
    u = ref.fcm_memberships(x, c, 5.0)
    np.testing.assert_array_equal(f.result_.labels.numpy(), u.argmax(1).numpy())


def test_fcm_explicit_fuzzifier():
    x = gaussian_blobs(2000, 2, 3, seed=1, dtype=torch.float64)
    cfg = tdc.ClusterConfig(n_clusters=3, max_iter=3, dtype="fp64", init="first_k", fuzzifier=2.0)
    f = tdc.FuzzyCMeans(cfg).fit(x)
    c = x[:3].clone()
    for _ in range(3):
        wx, ws, _ = ref.fcm_partial(x, c, 2.0)
        c = wx / ws[:, None]
    np.testing.assert_allclose(f.result_.centers, c.numpy(), rtol=1e-10)


def test_predict():
    x = gaussian_blobs(2000, 2, 4, seed=9, dtype=torch.float64)
    km = tdc.KMeans(tdc.ClusterConfig(n_clusters=4, max_iter=10, dtype="fp64")).fit(x)
    assert torch.equal(km.predict(x), km.result_.labels)


def test_config_validation():
    with pytest.raises(ValueError):
        tdc.ClusterConfig(n_clusters=0)
    with pytest.raises(ValueError):
        tdc.ClusterConfig(n_clusters=3, dtype="fp16")
    with pytest.raises(ValueError):
        tdc.ClusterConfig(n_clusters=3, init="bogus")
    with pytest.raises(ValueError):
        tdc.ClusterConfig(n_clusters=3, fcm_distances="bf16x9")
    assert tdc.ClusterConfig(n_clusters=3).fcm_distances == "x3"


def test_kmeans_parallel_init_quality():
    from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs as gb
    x = gb(30000, 3, 20, seed=4, dtype=torch.float64)
    res = {}
    for init in ("kmeans||", "random"):
        res[init] = tdc.KMeans(tdc.ClusterConfig(n_clusters=20, max_iter=0, dtype="fp64",
                                                 init=init, seed=2)).fit(x).result_.inertia
    assert res["kmeans||"] < 0.6 * res["random"]


def test_spherical_kmeans_matches_cosine_reference():
    g = torch.Generator().manual_seed(0)
    dirs = torch.nn.functional.normalize(torch.randn(6, 16, generator=g, dtype=torch.float64), dim=1)
    lab = torch.randint(0, 6, (6000,), generator=g)
    scale = torch.rand(6000, 1, generator=g, dtype=torch.float64) * 10 + 0.1  # norms must not matter
    x = (dirs[lab] + 0.05 * torch.randn(6000, 16, generator=g, dtype=torch.float64)) * scale
    r = tdc.KMeans(tdc.ClusterConfig(n_clusters=6, max_iter=15, dtype="fp64", spherical=True,
                                     init="kmeans++", seed=1)).fit(x).result_
    c = torch.as_tensor(r.centers)
    torch.testing.assert_close(c.norm(dim=1), torch.ones(6, dtype=torch.float64))
    cos = torch.nn.functional.normalize(x, dim=1) @ c.t()
    assert torch.equal(cos.argmax(1).to(torch.int32), r.labels)
    # every true direction is recovered by some centroid
    assert (dirs @ c.t()).max(1).values.min() > 0.99


def test_bounded_algorithm_falls_back_to_lloyd_on_cpu():
    x = gaussian_blobs(3000, 3, 5, seed=2, dtype=torch.float64)
    cfg = tdc.ClusterConfig(n_clusters=5, max_iter=8, dtype="fp64", seed=1)
    a = tdc.KMeans(cfg).fit(x).result_
    km = tdc.KMeans(cfg.replace(algorithm="bounded")).fit(x)
    assert not km.engine_.enabled
    np.testing.assert_array_equal(km.result_.centers, a.centers)
    with pytest.raises(ValueError):
        tdc.ClusterConfig(n_clusters=2, algorithm="elkan")


def test_fcm_predict_and_memberships_match_fit():
    import torch
    from tensorflow_distributed_clustering_amd import ClusterConfig, FuzzyCMeans
    g = torch.Generator().manual_seed(2)
    x = torch.randn(4000, 3, generator=g, dtype=torch.float64) + \
        torch.randint(0, 3, (4000, 1), generator=g).double() * 4
    fcm = FuzzyCMeans(ClusterConfig(n_clusters=3, max_iter=15, dtype="fp64", seed=1,
                                    fuzzifier=2.0)).fit(x)
    lab = fcm.predict(x)
    assert torch.equal(lab, fcm.result_.labels)
    u = fcm.memberships(x, chunk_rows=1000)
    assert u.shape == (4000, 3)
    torch.testing.assert_close(u.sum(1), torch.ones(4000, dtype=torch.float64))
    assert torch.equal(u.argmax(1).to(torch.int32), lab)



@pytest.mark.parametrize("method", ["kmeans", "fcm"])
def test_warmup_step_leaves_no_trace(method):
    """The untimed warm-up step (setup) restores the centroids and the iteration count:
    the steps after it match an engine that never warmed up."""
    from tensorflow_distributed_clustering_amd.models.fcm import FcmEngine
    from tensorflow_distributed_clustering_amd.models.kmeans import LloydEngine
    from tensorflow_distributed_clustering_amd.parallel.dist import init_comm
    comm = init_comm("cpu")
    x = gaussian_blobs(3000, 4, 6, seed=5, dtype=torch.float64)
    cfg = tdc.ClusterConfig(n_clusters=6, max_iter=5, dtype="fp64", seed=3, fuzzifier=2.0,
                            empty_cluster="reseed" if method == "kmeans" else "keep")
    Eng = LloydEngine if method == "kmeans" else FcmEngine
    a, b = Eng(x, cfg, comm, 3000, 0), Eng(x, cfg, comm, 3000, 0)
    c0 = a.C.clone()
    a.warmup(force=True)
    assert torch.equal(a.C, c0) and a.n_iter == 0
    for _ in range(3):
        a.step()
        b.step()
    assert torch.equal(a.C, b.C) and a.n_iter == b.n_iter == 3


def test_warmup_does_not_prepay_the_first_full_update():
    """After the untimed warm-up, timed iteration 1 is a FULL update (every row re-summed),
    as the reference's computation_time includes its first iteration's full work
    (`scripts/distribuitedClustering.py:277-280`), and the run matches a cold engine."""
    from tensorflow_distributed_clustering_amd.models.kmeans import LloydEngine
    from tensorflow_distributed_clustering_amd.parallel.dist import init_comm
    comm = init_comm("cpu")
    x = gaussian_blobs(3000, 4, 6, seed=5, dtype=torch.float64)
    cfg = tdc.ClusterConfig(n_clusters=6, max_iter=5, dtype="fp64", seed=3, update="delta",
                            delta_refresh=0)
    a, b = LloydEngine(x, cfg, comm, 3000, 0), LloydEngine(x, cfg, comm, 3000, 0)
    assert a.delta is not None
    a.warmup(force=True)
    s0 = a.update_stats()
    a.step()
    s1 = a.update_stats()
    assert s1["full_steps"] - s0["full_steps"] == 1, (s0, s1)
    for _ in range(2):
        a.step()
    for _ in range(3):
        b.step()
    torch.testing.assert_close(a.C, b.C)
    assert a.update_stats()["full_steps"] - s0["full_steps"] == b.update_stats()["full_steps"]
