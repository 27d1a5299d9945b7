"""Native deterministic update (ClusterConfig.deterministic): fixed-point int64
partial sums (ops.NativeUpdate) against an exact PyTorch int64 reference of the same op,
bitwise run-to-run reproducibility of whole fits (full and delta updates), and agreement
with the float update.  Reference analogue: the per-GPU segment sums,
notebooks/visualization.ipynb:260-264."""
import numpy as np
import pytest
import torch

import tensorflow_distributed_clustering_amd as tdc
from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
from tensorflow_distributed_clustering_amd.ops import DC_NEXT, DC_WORDS, fixed_point_scale

pytestmark = pytest.mark.gpu


def _ops():
    from tensorflow_distributed_clustering_amd import _native
    return _native.require()


@pytest.mark.parametrize("xdt", [torch.bfloat16, torch.float32, torch.float64])
@pytest.mark.parametrize("n,d,k", [(60_001, 128, 1024), (7000, 33, 50)])
def test_fixed_point_update_exact(gpu, xdt, n, d, k):
    """int64 sums equal sum_i rint(x_i * 2^S) exactly (any order of the atomics)."""
    ops = _ops()
    g = torch.Generator().manual_seed(d + k)
    x = (torch.randn(n, d, generator=g, dtype=torch.float64) * 4).to(xdt).to(gpu)
    lab = torch.randint(0, k, (n,), generator=g, dtype=torch.int32).to(gpu)
    scale = fixed_point_scale(float(x.abs().max()), n, elem32=xdt != torch.float64)
    sums = torch.zeros(k, d, dtype=torch.int64, device=gpu)
    counts = torch.zeros(k, dtype=torch.int64, device=gpu)
    work = torch.zeros(int(ops.update_sorted_workspace(n, k)), dtype=torch.int32, device=gpu)
    ops.update_sorted(x, lab, sums, counts, work, None, None, None, scale)
    fx = (x.double() * scale).round().long()  # round half to even, as v_rndne / int64 rn
    rs = torch.zeros(k, d, dtype=torch.int64, device=gpu).index_add_(0, lab.long(), fx)
    assert torch.equal(sums, rs)
    assert torch.equal(counts, torch.bincount(lab.long(), minlength=k))
    # the delta update in fixed point: +x at new, -x at old, exactly
    prev = lab.clone()
    new = lab.clone()
    mv = torch.rand(n, generator=g) < 0.1
    new[mv.to(gpu)] = torch.randint(0, k, (int(mv.sum()),), generator=g,
                                    dtype=torch.int32).to(gpu)
    dwork = torch.zeros(int(ops.delta_workspace(n, k)), dtype=torch.int32, device=gpu)
    ctrl = torch.zeros(DC_WORDS, dtype=torch.int32, device=gpu)
    ctrl[DC_NEXT] = 0
    sums.zero_()
    counts.zero_()
    ops.delta_update(x, new, prev, sums, counts, dwork, ctrl, None, None, None, None, scale)
    i = torch.nonzero(new != lab).flatten()
    rs = torch.zeros(k, d, dtype=torch.int64, device=gpu)
    rs.index_add_(0, new.long()[i], fx[i]).index_add_(0, lab.long()[i], -fx[i])
    assert torch.equal(sums, rs)


@pytest.mark.parametrize("update", ["full", "delta"])
def test_deterministic_fit_bitwise_reproducible(gpu, update):
    """Headline-like shape: two fits give identical centroids and labels, and they agree
    with the float update."""
    n, d, k = 500_000, 128, 1024
    x = gaussian_blobs(n, d, k, seed=12, dtype=torch.bfloat16, device=gpu)
    cfg = tdc.ClusterConfig(n_clusters=k, max_iter=8, dtype="bf16", seed=2, deterministic=True,
                            update=update)
    runs = [tdc.KMeans(cfg, device=gpu).fit(x) for _ in range(2)]
    a, b = runs[0].result_, runs[1].result_
    assert runs[0].engine_.fixed and runs[0].engine_.buf.dtype == torch.int64
    assert runs[0].engine_.update_mode == update
    assert np.array_equal(a.centers, b.centers)
    assert torch.equal(a.labels, b.labels)
    f = tdc.KMeans(cfg.replace(deterministic=False), device=gpu).fit(x).result_
    # the float update's sums differ in the last bits; a bf16 near tie that flips one row
    # moves its two centroids by ~|x - c| / count, so compare per centroid
    ok = np.isclose(a.centers, f.centers, rtol=1e-5, atol=1e-5).all(1)
    assert ok.mean() >= 0.99, ok.mean()
    assert (a.labels == f.labels).float().mean().item() > 0.999


@pytest.mark.parametrize("dtype,d,k", [("fp32", 40, 64), ("fp64", 20, 30), ("fp8", 256, 128)])
def test_deterministic_other_dtypes(gpu, dtype, d, k):
    tdt = {"fp32": torch.float32, "fp64": torch.float64, "fp8": torch.bfloat16}[dtype]
    x = gaussian_blobs(80_000, d, k, seed=5, dtype=tdt, device=gpu)
    cfg = tdc.ClusterConfig(n_clusters=k, max_iter=6, dtype=dtype, seed=3, deterministic=True)
    a = tdc.KMeans(cfg, device=gpu).fit(x).result_
    b = tdc.KMeans(cfg, device=gpu).fit(x).result_
    assert np.array_equal(a.centers, b.centers)
    f = tdc.KMeans(cfg.replace(deterministic=False), device=gpu).fit(x).result_
    tol = 1e-9 if dtype == "fp64" else 1e-5
    np.testing.assert_allclose(a.centers, f.centers, rtol=tol, atol=tol)


@pytest.mark.parametrize("xdt", [torch.float32, torch.float64])
def test_deterministic_mixed_scale_unbiased(gpu, xdt):
    """One feature ~1e4, the others ~3e-2: the fixed-point step follows the global max |x|,
    so the small features are many steps of rounding each; rounded to nearest the errors
    average out (round-toward-zero biased every small positive element by half a step:
    ~1e-3 relative on their means).  fp64 rows use the finer sum-bound step."""
    ops = _ops()
    n, d, k = 200_000, 8, 4
    g = torch.Generator().manual_seed(1)
    x = torch.randn(n, d, generator=g, dtype=torch.float64) * 1e-2 + 0.03
    x[:, 0] = torch.randn(n, generator=g, dtype=torch.float64) * 1e4
    x = x.to(xdt).to(gpu)
    lab = torch.randint(0, k, (n,), generator=g, dtype=torch.int32).to(gpu)
    scale = fixed_point_scale(float(x.abs().max()), n, elem32=xdt != torch.float64)
    sums = torch.zeros(k, d, dtype=torch.int64, device=gpu)
    counts = torch.zeros(k, dtype=torch.int64, device=gpu)
    work = torch.zeros(int(ops.update_sorted_workspace(n, k)), dtype=torch.int32, device=gpu)
    ops.update_sorted(x, lab, sums, counts, work, None, None, None, scale)
    means = (sums.double() / scale) / counts.double()[:, None]
    rs = torch.zeros(k, d, dtype=torch.float64, device=gpu).index_add_(0, lab.long(), x.double())
    ref = rs / torch.bincount(lab.long(), minlength=k).double()[:, None]
    rel = ((means - ref).abs() / ref.abs())[:, 1:].max().item()
    assert rel < (2e-5 if xdt == torch.float32 else 2e-8), rel


def test_fixed_point_scale_rejects_non_finite():
    import math
    with pytest.raises(ValueError, match="NaN or an infinity"):
        fixed_point_scale(math.inf, 10)
    with pytest.raises(ValueError):
        fixed_point_scale(float("nan"), 10)
