"""Serving API on CPU (torch backend): ClusterPredictor, KMeans.predict/score,
MiniBatchKMeans.partial_fit (online updates)."""
import numpy as np
import torch

import tensorflow_distributed_clustering_amd as tdc
from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
from tensorflow_distributed_clustering_amd.ops import reference as ref
from tensorflow_distributed_clustering_amd.serving import ClusterPredictor


def test_predictor_matches_reference_assign():
    x = gaussian_blobs(3000, 7, 12, seed=2, dtype=torch.float64)
    c = x[torch.randperm(3000, generator=torch.Generator().manual_seed(0))[:12]].clone()
    p = ClusterPredictor(c.numpy(), dtype="fp64", device="cpu")
    lab, d2 = p.predict(x, return_distance=True)
    rlab, rd2 = ref.assign(x, c, exact=True)
    assert torch.equal(lab.long(), rlab.long())
    torch.testing.assert_close(d2.double(), rd2.double(), rtol=1e-12, atol=1e-12)
    assert abs(p.score(x) + float(rd2.sum())) < 1e-6 * float(rd2.sum())
    # outputs are copies: a second request does not overwrite the first answer
    lab2 = p.predict(x[:3000].flip(0))
    assert torch.equal(lab.long(), rlab.long()) and lab2.shape == lab.shape
    assert p.predict(x[:0]).numel() == 0


def test_kmeans_predict_and_score_on_training_rows():
    x = gaussian_blobs(4000, 3, 6, seed=5, dtype=torch.float64)
    km = tdc.KMeans(tdc.ClusterConfig(n_clusters=6, max_iter=15, dtype="fp64", seed=1)).fit(x)
    assert torch.equal(km.predict(x).long(), km.result_.labels.long())
    assert abs(km.score(x) + km.result_.inertia) <= 1e-9 * km.result_.inertia


def test_minibatch_partial_fit_online():
    x = gaussian_blobs(40000, 4, 8, seed=9, dtype=torch.float32)
    cfg = tdc.ClusterConfig(n_clusters=8, dtype="fp32", seed=3, init="kmeans++")
    mb = tdc.MiniBatchKMeans(cfg)
    g = torch.Generator().manual_seed(1)
    for _ in range(30):
        mb.partial_fit(x[torch.randint(40000, (2048,), generator=g)])
    assert mb.engine_.n_iter == 30
    c = mb.cluster_centers_
    assert c.shape == (8, 4) and np.isfinite(c).all()
    full = tdc.KMeans(tdc.ClusterConfig(n_clusters=8, max_iter=30, dtype="fp32", seed=3,
                                        init="kmeans++")).fit(x)
    _, md = ref.assign(x.double(), torch.as_tensor(c), exact=True)
    assert float(md.sum()) <= 1.10 * full.result_.inertia
    lab = mb.predict(x[:100])
    assert lab.shape == (100,) and int(lab.max()) < 8
