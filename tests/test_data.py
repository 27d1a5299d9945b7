"""Data layer: array_split sharding, world-size-invariant synthetic data, NPZ memory map."""
import numpy as np
import pytest
import torch

from tensorflow_distributed_clustering_amd.data.npz import load_shard, open_npz_member
from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs, make_data
from tensorflow_distributed_clustering_amd.parallel.dist import shard_bounds, shard_sizes


@pytest.mark.parametrize("n,w", [(10, 3), (25, 8), (7, 7), (3, 5), (1000003, 8)])
def test_shard_bounds_is_array_split(n, w):
    ref = [len(a) for a in np.array_split(np.arange(n), w)]
    assert shard_sizes(n, w) == ref
    starts = [shard_bounds(n, w, r)[0] for r in range(w)]
    assert starts == list(np.cumsum([0] + ref[:-1]))


def test_blobs_world_invariant():
    full = gaussian_blobs(1000, 7, 5, seed=3)
    parts = [gaussian_blobs(e - s, 7, 5, seed=3, row_offset=s)
             for s, e in (shard_bounds(1000, 3, r) for r in range(3))]
    assert torch.equal(torch.cat(parts), full)
    small_chunks = gaussian_blobs(1000, 7, 5, seed=3, chunk_rows=17)
    assert torch.equal(small_chunks, full)


def test_blobs_statistics():
    x, y = gaussian_blobs(200000, 4, 3, seed=1, cluster_std=2.0, return_labels=True)
    assert set(y.unique().tolist()) == {0, 1, 2}
    from tensorflow_distributed_clustering_amd.data.synth import blob_centers
    c = torch.as_tensor(blob_centers(3, 4, 1), dtype=torch.float32)
    resid = x - c[y.long()]
    assert abs(float(resid.mean())) < 0.02
    assert abs(float(resid.std()) - 2.0) < 0.02


def test_npz_mmap_roundtrip(tmp_path):
    p = str(tmp_path / "d.npz")
    make_data(p, 5000, 5, 1826273)
    x = open_npz_member(p, "X")
    with np.load(p) as z:
        np.testing.assert_array_equal(np.asarray(x), z["X"])
        assert z["X"].dtype == np.float64 and set(np.unique(z["Y"])) <= {0, 1}
    parts = [load_shard(p, r, 3) for r in range(3)]
    np.testing.assert_array_equal(np.concatenate([a for a, _, _ in parts]), z_x(p))
    assert [o for _, _, o in parts] == [0, 1667, 3334]


def z_x(p):
    with np.load(p) as z:
        return z["X"]


def test_make_classification_matches_reference_call():
    from sklearn.datasets import make_classification
    from tensorflow_distributed_clustering_amd.data.synth import make_classification_compat
    X, Y = make_classification_compat(1000, 5, 1826273)
    X2, Y2 = make_classification(n_samples=1000, n_features=5, n_informative=5, n_redundant=0,
                                 n_classes=2, n_clusters_per_class=1, shuffle=True,
                                 random_state=1826273)
    np.testing.assert_array_equal(X, X2)
    np.testing.assert_array_equal(Y, Y2)
