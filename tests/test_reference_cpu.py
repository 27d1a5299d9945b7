"""Reference-op semantics (CPU, fp64): the oracle the HIP kernels are tested against.

Semantics from the reference engine: first-minimum argmin, per-cluster
sums/counts, FCM with d^(-2/(m-1)) memberships, NaN->0 guard, u^m weights.
"""
import numpy as np
import pytest
import torch

from tensorflow_distributed_clustering_amd.ops import reference as ref


def _np_kmeans_step(x, c):
    d = ((x[:, None, :] - c[None]) ** 2).sum(-1)
    lab = d.argmin(1)
    k = c.shape[0]
    sums = np.zeros_like(c)
    np.add.at(sums, lab, x)
    counts = np.bincount(lab, minlength=k).astype(np.float64)
    return lab, d.min(1), sums, counts


def test_assign_matches_numpy_and_ties_first_index():
    rng = np.random.default_rng(0)
    x = rng.normal(size=(500, 5))
    c = rng.normal(size=(7, 5))
    c[4] = c[2]  # duplicate centroid -> tie -> first index (TF ArgMin)
    lab, md = ref.assign(torch.from_numpy(x), torch.from_numpy(c), exact=True)
    nl, nd, _, _ = _np_kmeans_step(x, c)
    assert np.array_equal(lab.numpy(), nl)
    assert not (lab.numpy() == 4).any()
    np.testing.assert_allclose(md.numpy(), nd, rtol=1e-12)


def test_expanded_vs_exact_distance():
    rng = np.random.default_rng(1)
    x = torch.from_numpy(rng.normal(size=(300, 16)))
    c = torch.from_numpy(rng.normal(size=(9, 16)))
    torch.testing.assert_close(ref.pairwise_sqdist(x, c, False), ref.pairwise_sqdist(x, c, True))


def test_cluster_sums_and_chunking():
    rng = np.random.default_rng(2)
    x = rng.normal(size=(1000, 3))
    c = rng.normal(size=(4, 3))
    lab, _ = ref.assign(torch.from_numpy(x), torch.from_numpy(c), exact=True, chunk_elems=37)
    nl, _, nsums, ncounts = _np_kmeans_step(x, c)
    assert np.array_equal(lab.numpy(), nl)
    s, n = ref.cluster_sums(torch.from_numpy(x), lab, 4)
    np.testing.assert_allclose(s.numpy(), nsums, rtol=1e-12)
    np.testing.assert_array_equal(n.numpy(), ncounts)


@pytest.mark.parametrize("policy,expect", [("keep", "old"), ("nan", "nan"), ("zero", 0.0)])
def test_empty_cluster_policies(policy, expect):
    sums = torch.tensor([[2.0, 4.0], [0.0, 0.0]], dtype=torch.float64)
    counts = torch.tensor([2.0, 0.0], dtype=torch.float64)
    old = torch.tensor([[9.0, 9.0], [5.0, 6.0]], dtype=torch.float64)
    new = ref.finalize(sums, counts, old, policy)
    assert new[0].tolist() == [1.0, 2.0]
    if expect == "old":
        assert new[1].tolist() == [5.0, 6.0]
    elif expect == "nan":
        assert torch.isnan(new[1]).all()
    else:
        assert new[1].tolist() == [0.0, 0.0]


def test_fcm_matches_closed_form():
    rng = np.random.default_rng(3)
    x = rng.normal(size=(200, 5))
    c = rng.normal(size=(3, 5))
    m = 5.0  # the reference's m := D
    d = np.sqrt(((x[:, None] - c[None]) ** 2).sum(-1))
    t = d ** (-2.0 / (m - 1.0))
    u = t / t.sum(1, keepdims=True)
    w = u ** m
    wx, ws, lab = ref.fcm_partial(torch.from_numpy(x), torch.from_numpy(c), m)
    np.testing.assert_allclose(wx.numpy(), w.T @ x, rtol=1e-10)
    np.testing.assert_allclose(ws.numpy(), w.sum(0), rtol=1e-10)
    np.testing.assert_array_equal(lab.numpy(), u.argmax(1))


def test_fcm_point_on_centroid_nan_guard():
    c = torch.tensor([[0.0, 0.0], [3.0, 0.0]], dtype=torch.float64)
    x = torch.tensor([[0.0, 0.0], [1.0, 0.0]], dtype=torch.float64)
    u_compat = ref.fcm_memberships(x, c, 2.0, nan_to_zero=True)
    assert u_compat[0].tolist() == [0.0, 0.0]  # reference: NaN -> 0 everywhere
    u_fixed = ref.fcm_memberships(x, c, 2.0, nan_to_zero=False)
    assert u_fixed[0].tolist() == [1.0, 0.0]
    assert abs(float(u_fixed[1].sum()) - 1.0) < 1e-12


def test_fcm_rejects_m_le_1():
    x = torch.zeros(3, 1, dtype=torch.float64)
    with pytest.raises(ValueError):
        ref.fcm_memberships(x, x[:2], 1.0)


def test_kmeanspp_oracle_picks_distinct_far_points():
    g = torch.Generator().manual_seed(0)
    blobs = torch.cat([torch.randn(100, 2, generator=g, dtype=torch.float64) * 0.1 + o
                       for o in (torch.tensor([0.0, 0.0]), torch.tensor([50.0, 0.0]),
                                 torch.tensor([0.0, 50.0]))])
    c = ref.kmeanspp(blobs, 3, g)
    # one center per well-separated blob
    owner = ((c[:, None, :] - torch.tensor([[0.0, 0.0], [50.0, 0.0], [0.0, 50.0]],
                                           dtype=torch.float64)[None]) ** 2).sum(-1).argmin(1)
    assert sorted(owner.tolist()) == [0, 1, 2]
