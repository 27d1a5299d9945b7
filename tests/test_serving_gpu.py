"""Serving on the GPU: ClusterPredictor on the bf16 MFMA / fp8 / fp64 kernels, layout
copy vs in-layout input, hipGraph replay, MiniBatchKMeans.partial_fit."""
import numpy as np
import pytest
import torch

import tensorflow_distributed_clustering_amd as tdc
from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
from tensorflow_distributed_clustering_amd.ops import reference as ref
from tensorflow_distributed_clustering_amd.serving import ClusterPredictor

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype,d,k", [("bf16", 128, 1024), ("bf16", 100, 64), ("fp8", 768, 256),
                                       ("fp64", 5, 3)])
def test_predictor_gpu(gpu, dtype, d, k):
    x = gaussian_blobs(50_000, d, k, seed=3, dtype=torch.float32, device=gpu)
    c = x[:: 50_000 // k][:k].double().cpu().numpy()
    p = ClusterPredictor(c, dtype=dtype, device=gpu)
    assert p.backend != "torch"
    xin = x.to(torch.bfloat16) if dtype == "bf16" and d == 128 else x
    lab, d2 = p.predict(xin, return_distance=True)
    # near-tie tolerant check against the fp64 oracle
    dd = ref.pairwise_sqdist(x.double(), torch.as_tensor(c, device=gpu), exact=True)
    best = dd.min(1).values
    got = dd.gather(1, lab.long()[:, None]).squeeze(1)
    tol = {"fp64": 1e-9, "bf16": 3e-2, "fp8": 0.15}[dtype]  # e4m3: 3 mantissa bits
    assert int(((got - best) > tol * (best.abs() + (x.double() ** 2).sum(1))).sum()) == 0
    # graph replay == eager for the same size
    p.capture(x.shape[0])
    lab_g, d2_g = p.predict(x, return_distance=True)
    assert torch.equal(lab_g, lab if xin is x else p.predict(x.to(xin.dtype)))
    assert torch.isfinite(d2_g).all()


def test_kmeans_predict_gpu_bf16(gpu):
    x = gaussian_blobs(200_000, 64, 128, seed=4, dtype=torch.bfloat16, device=gpu)
    km = tdc.KMeans(tdc.ClusterConfig(n_clusters=128, max_iter=5, dtype="bf16", seed=1),
                    device=gpu).fit(x)
    agree = (km.predict(x) == km.result_.labels).float().mean().item()
    assert agree > 0.999  # same kernel, same centres (fp32 round trip of the centres)


def test_minibatch_partial_fit_gpu(gpu):
    x = gaussian_blobs(400_000, 128, 64, seed=8, dtype=torch.bfloat16, device=gpu)
    cfg = tdc.ClusterConfig(n_clusters=64, dtype="bf16", seed=2, init="kmeans++")
    mb = tdc.MiniBatchKMeans(cfg, device=gpu)
    g = torch.Generator(device=gpu).manual_seed(0)
    for _ in range(20):  # the first batch seeds k-means++: large enough to see every blob
        mb.partial_fit(x[torch.randint(400_000, (65536,), generator=g, device=gpu)])
    full = tdc.KMeans(tdc.ClusterConfig(n_clusters=64, max_iter=20, dtype="bf16", seed=2,
                                        init="kmeans++"), device=gpu).fit(x)
    _, md = ref.assign(x.double(), torch.as_tensor(mb.cluster_centers_, device=gpu), exact=True)
    assert float(md.sum()) <= 1.10 * full.result_.inertia


@pytest.mark.parametrize("dtype,d", [("fp8", 768), ("bf16", 384)])
def test_predictor_reused_buffer_requantised(gpu, dtype, d):
    """Two requests of the same size with different rows: the per-size layout buffer is
    refilled in place, so derived operands (fp8 quantisation, row norms) must be redone."""
    k = 64
    x = gaussian_blobs(20_000, d, k, seed=1, dtype=torch.float32, device=gpu)
    c = x[:k].double().cpu().numpy()
    p = ClusterPredictor(c, dtype=dtype, device=gpu)
    a, b = x[:10_000], x[10_000:]
    la = p.predict(a)
    lb = p.predict(b)
    fresh = ClusterPredictor(c, dtype=dtype, device=gpu)
    assert torch.equal(lb, fresh.predict(b))
    assert torch.equal(la, fresh.predict(a))


def test_fcm_predict_gemm_path(gpu):
    """FuzzyCMeans.predict at D > 16 runs the MFMA FCM tower and reproduces the fit's label
    pass."""
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
    x = gaussian_blobs(50000, 64, 32, seed=4, dtype=torch.float32, device=gpu)
    fcm = tdc.FuzzyCMeans(tdc.ClusterConfig(n_clusters=32, max_iter=3, dtype="bf16", seed=1,
                                            fuzzifier=2.0)).fit(x)
    assert fcm.result_.backend == "hip_fcm_mfma"
    lab = fcm.predict(x)
    assert (lab == fcm.result_.labels).float().mean().item() > 0.999
    u = fcm.memberships(x[:1000])
    assert (u.argmax(1).to(torch.int32) == lab[:1000]).float().mean().item() > 0.99
