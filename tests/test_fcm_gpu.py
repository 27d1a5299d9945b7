"""Native FCM towers against the fp64 PyTorch oracle (``ops/reference.fcm_partial``, the
reference's op chain `scripts/distribuitedClustering.py:108-137`).

* ``fcm_tower_*`` (csrc/fcm_tower.hip): fp32/fp64, any K, D <= 256, exact difference-form
  distances -- the path of every shape fcm_small does not cover;
* ``fcm_mfma_*`` (csrc/fcm_mfma.hip): fp32 on bf16 matrix cores with hi/lo split operands.

Each case includes a point exactly on a centroid (the NaN -> 0 guard, or the one-hot limit
with ``nan_to_zero=False``) and a ragged N.
"""
import pytest
import torch

from tensorflow_distributed_clustering_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _data(n, k, d, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, d, generator=g, dtype=torch.float64)
    c = x[torch.randperm(n, generator=g)[:k]] + 0.05 * torch.randn(k, d, generator=g,
                                                                   dtype=torch.float64)
    x[7] = c[min(3, k - 1)]  # a point exactly on a centroid
    return x, c


def _check(wx, ws, lab, x, c, m, nz, rtol, agree):
    # exact difference form: a point ON a centroid is at distance exactly 0
    a, b, lr = ref.fcm_partial(x.double(), c.double(), m, nz, exact=True)
    cen = wx / ws.clamp_min(1e-300)[:, None]
    cen_ref = a / b.clamp_min(1e-300)[:, None]
    ok = b > 1e-12 * b.max()
    torch.testing.assert_close(ws[ok], b[ok], rtol=rtol, atol=rtol * float(b.max()) * 1e-3)
    torch.testing.assert_close(cen[ok], cen_ref[ok], rtol=rtol, atol=rtol)
    assert (lab.long().cpu() == lr.long().cpu()).double().mean().item() >= agree


@pytest.mark.parametrize("dt", [torch.float64, torch.float32])
@pytest.mark.parametrize("k,d", [(32, 5), (20, 9), (100, 3), (64, 40), (300, 17), (129, 128),
                                 (50, 256), (1000, 12)])
@pytest.mark.parametrize("m", [2.0, 2.5])
@pytest.mark.parametrize("nz", [True, False])
def test_fcm_tower_matches_oracle(gpu, dt, k, d, m, nz):
    from tensorflow_distributed_clustering_amd import _native
    ops = _native.require()
    n = 6001 if k * d > 20000 else 20011
    x, c = _data(n, k, d, k * 7 + d)
    xg, cg = x.to(dt).to(gpu), c.to(dt).to(gpu)
    lab = torch.empty(n, dtype=torch.int32, device=gpu)
    ri = torch.empty(n, dtype=dt, device=gpu)
    wx = torch.zeros(k, d, dtype=torch.float64, device=gpu)
    ws = torch.zeros(k, dtype=torch.float64, device=gpu)
    ops.fcm_tower_stats(xg, cg, m, nz, lab, ri)
    ops.fcm_tower_accum(xg, cg, m, nz, ri, wx, ws)
    rtol = 1e-9 if dt == torch.float64 else 2e-4 * m
    _check(wx.cpu(), ws.cpu(), lab, xg.cpu(), cg.cpu(), m, nz, rtol,
           0.99999 if dt == torch.float64 else 0.999)


@pytest.mark.parametrize("k,d", [(32, 17), (100, 64), (257, 128), (1024, 128), (130, 33),
                                 (64, 128)])
@pytest.mark.parametrize("m", [2.0, 3.0, 1.5])
@pytest.mark.parametrize("nz", [True, False])
def test_fcm_mfma_matches_oracle(gpu, k, d, m, nz):
    from tensorflow_distributed_clustering_amd.ops import HipMfmaFCM
    n = 20001
    x, c = _data(n, k, d, k + d)
    xg, cg = x.float().to(gpu), c.float().to(gpu)
    ops = HipMfmaFCM(xg, k, m, nz)
    lab = torch.empty(n, dtype=torch.int32, device=gpu)
    wx = torch.zeros(k, d, dtype=torch.float64, device=gpu)
    ws = torch.zeros(k, dtype=torch.float64, device=gpu)
    ops.step(cg, lab, wx, ws)
    # bf16x3 distances: |d2 error| ~ 2^-17 (|x|^2 + |c|^2), relative to the small d2 of a
    # point next to its centroid (|x|^2 / d2 ~ 400 here) -> ~0.1 % per (m - 1) in t
    _check(wx.cpu(), ws.cpu(), lab, xg.cpu(), cg.cpu(), m, nz, 2e-3 * m, 0.998)
    lab2 = torch.empty_like(lab)
    ops.assign(cg, lab2)
    assert torch.equal(lab, lab2)


@pytest.mark.parametrize("k,d", [(33, 256), (257, 384), (1024, 768), (100, 1024), (64, 200)])
@pytest.mark.parametrize("m", [2.0, 1.5, 3.0])
@pytest.mark.parametrize("nz", [True, False])
def test_fcm_mfma_wide_matches_oracle(gpu, k, d, m, nz):
    """fp32, 128 < D <= 1024 on the matrix cores (distance GEMM into the row block, the
    row pass, W^T X GEMM), over several chunks with a ragged tail, against the fp64 oracle
    with the register MFMA tower's tolerances."""
    from tensorflow_distributed_clustering_amd.ops import HipMfmaWideFCM
    n = 9001
    x, c = _data(n, k, d, 5 * k + d)
    xg, cg = x.float().to(gpu), c.float().to(gpu)
    ops = HipMfmaWideFCM(xg, k, m, nz)
    ops.chunk_elems = 4000 * k
    lab = torch.empty(n, dtype=torch.int32, device=gpu)
    wx = torch.zeros(k, d, dtype=torch.float64, device=gpu)
    ws = torch.zeros(k, dtype=torch.float64, device=gpu)
    ops.step(cg, lab, wx, ws)
    _check(wx.cpu(), ws.cpu(), lab, xg.cpu(), cg.cpu(), m, nz, 2e-3 * m, 0.998)
    lab2 = torch.full_like(lab, -1)
    ops.assign(cg, lab2)
    assert torch.equal(lab, lab2)


@pytest.mark.parametrize("k,d,m", [(32, 20, 8.0), (64, 24, 12.0), (48, 33, 10.0)])
@pytest.mark.parametrize("nz", [True, False])
def test_fcm_mfma_large_fuzzifier(gpu, k, d, m, nz):
    """Large fuzzifiers on the MFMA tower: the bf16x3 distance error enters
    t = d^(-2/(m-1)) scaled by 2/(m-1), so w = u^m carries ~2m/(m-1) ~ 2x the distance
    error however large m is -- the m = 2 tolerance holds (no m-proportional slack)."""
    from tensorflow_distributed_clustering_amd.ops import HipMfmaFCM
    n = 20001
    x, c = _data(n, k, d, 3 * k + d)
    xg, cg = x.float().to(gpu), c.float().to(gpu)
    ops = HipMfmaFCM(xg, k, m, nz)
    lab = torch.empty(n, dtype=torch.int32, device=gpu)
    wx = torch.zeros(k, d, dtype=torch.float64, device=gpu)
    ws = torch.zeros(k, dtype=torch.float64, device=gpu)
    ops.step(cg, lab, wx, ws)
    _check(wx.cpu(), ws.cpu(), lab, xg.cpu(), cg.cpu(), m, nz, 4e-3, 0.998)


@pytest.mark.parametrize("d,k,backend", [(20, 32, "hip_fcm_mfma"), (24, 40, "hip_fcm_tower")])
def test_fcm_fit_reference_fuzzifier_m_equals_d(gpu, d, k, backend):
    """fuzzifier=None (the reference's m = D) with dtype bf16: while the typical weight
    K^-m stays in fp32's range (D=20, K=32: 2^-100) the fit runs on the MFMA tower; past it
    (D=24, K=40: 2^-128, where every fp32 sum of u^m flushes to 0) the engine computes in
    fp64 (exact tower).  Both follow the fp64 torch fit."""
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.data.synth import blob_centers, gaussian_blobs
    x = gaussian_blobs(30000, d, k, seed=4, dtype=torch.float64, device=gpu)
    c0 = blob_centers(k, d, 4) + 0.3
    cfg = tdc.ClusterConfig(n_clusters=k, max_iter=4, dtype="bf16", init="given")
    r = tdc.FuzzyCMeans(cfg).fit(x, init_centers_=c0).result_
    assert r.backend == backend
    o = tdc.FuzzyCMeans(cfg.replace(dtype="fp64", backend="torch"),
                        device="cpu").fit(x.cpu(), init_centers_=c0).result_
    tol = 3e-3 if backend == "hip_fcm_mfma" else 1e-8
    torch.testing.assert_close(torch.as_tensor(r.centers), torch.as_tensor(o.centers),
                               rtol=tol, atol=tol)


@pytest.mark.parametrize("dtype", ["fp64", "fp32", "bf16"])
@pytest.mark.parametrize("k,d", [(100, 384), (257, 768), (40, 300), (1030, 1024)])
@pytest.mark.parametrize("nz", [True, False])
def test_fcm_wide_matches_oracle(gpu, dtype, k, d, nz):
    """D > 256 (past the register towers): the native wide tower -- exact difference-form
    distances of a row chunk into [rows, K], memberships in place, W^T X -- against the fp64
    oracle, over several chunks with a ragged tail (a point exactly on a centroid included).
    fp64 / fp32 are the exact tower (fp32 at the fp32 tolerance); bf16 selects the wide
    MFMA path (bf16x3 distances, bf16 weights), at its own tolerance."""
    from tensorflow_distributed_clustering_amd.ops import (HipMfmaWideFCM, HipWideFCM,
                                                            make_fcm_ops)
    n = 6001
    m = 2.0 if d != 300 else 3.0
    x, c = _data(n, k, d, k * 3 + d)
    dt = torch.float64 if dtype == "fp64" else torch.float32
    xg, cg = x.to(dt).to(gpu), c.to(dt).to(gpu)
    ops = make_fcm_ops(xg, k, dtype, m, nz)
    assert isinstance(ops, HipMfmaWideFCM if dtype == "bf16" else HipWideFCM)
    ops.chunk_elems = 2500 * k  # 3 chunks, the last ragged
    lab = torch.empty(n, dtype=torch.int32, device=gpu)
    wx = torch.zeros(k, d, dtype=torch.float64, device=gpu)
    ws = torch.zeros(k, dtype=torch.float64, device=gpu)
    ops.step(cg, lab, wx, ws)
    if dtype == "fp64":
        _check(wx.cpu(), ws.cpu(), lab, xg.cpu(), cg.cpu(), m, nz, 1e-9, 0.99999)
    elif dtype == "fp32":
        _check(wx.cpu(), ws.cpu(), lab, xg.cpu(), cg.cpu(), m, nz, 2e-4 * m, 0.999)
    else:  # bf16x3 distances, bf16 weights, as the register MFMA tower
        _check(wx.cpu(), ws.cpu(), lab, xg.cpu(), cg.cpu(), m, nz, 2e-3 * m, 0.998)
    lab2 = torch.full_like(lab, -1)
    ops.assign(cg, lab2)
    assert torch.equal(lab, lab2)


def test_fcm_dispatch_native_up_to_1024(gpu):
    """No GPU FCM shape up to D = 1024 falls back to a library GEMM or plain PyTorch."""
    from tensorflow_distributed_clustering_amd.ops import make_fcm_ops
    for dtype in ("fp32", "fp64", "bf16"):
        for d in (3, 17, 100, 200, 256, 300, 512, 768, 1024):
            for k in (3, 40, 300):
                ops = make_fcm_ops(torch.zeros(64, d, device=gpu), k, dtype, 2.0)
                assert ops.name.startswith("hip_fcm_"), (dtype, d, k, ops.name)


@pytest.mark.parametrize("dtype,d,k,backend", [("fp64", 5, 32, "hip_fcm_small"),
                                               ("fp64", 5, 40, "hip_fcm_small"),
                                               ("fp64", 384, 50, "hip_fcm_wide"),
                                               ("bf16", 512, 64, "hip_fcm_mfma"),
                                               ("bf16", 768, 40, "hip_fcm_mfma"),
                                               ("fp32", 512, 64, "hip_fcm_wide"),
                                               ("fp64", 6, 40, "hip_fcm_tower"),
                                               ("fp64", 64, 100, "hip_fcm_wide"),
                                               ("fp32", 12, 64, "hip_fcm_tower"),
                                               ("fp32", 128, 256, "hip_fcm_wide"),
                                               ("fp64", 128, 256, "hip_fcm_wide"),
                                               ("fp32", 64, 100, "hip_fcm_wide"),
                                               ("fp32", 32, 100, "hip_fcm_tower"),
                                               ("fp64", 32, 40, "hip_fcm_tower"),
                                               ("bf16", 128, 256, "hip_fcm_mfma")])
def test_fcm_fit_native_backends(gpu, dtype, d, k, backend):
    """Every FCM shape class runs a native backend and follows the fp64 torch fit."""
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.data.synth import blob_centers, gaussian_blobs
    x = gaussian_blobs(30000, d, k, seed=2, dtype=torch.float64, device=gpu)
    # one start per blob, off its centre: two centroids sharing a blob split along a
    # direction any rounding difference decides (a symmetric saddle), and a start ON a
    # data row is the reference's discontinuous NaN -> 0 case
    c0 = blob_centers(k, d, 2) + 0.3
    cfg = tdc.ClusterConfig(n_clusters=k, max_iter=4, dtype=dtype, init="given", fuzzifier=2.0)
    r = tdc.FuzzyCMeans(cfg).fit(x, init_centers_=c0).result_
    assert r.backend == backend
    o = tdc.FuzzyCMeans(cfg.replace(dtype="fp64", backend="torch"),
                        device="cpu").fit(x.cpu(), init_centers_=c0).result_
    tol = {"fp64": 1e-8, "fp32": 1e-4, "bf16": 3e-3}[dtype]
    torch.testing.assert_close(torch.as_tensor(r.centers), torch.as_tensor(o.centers),
                               rtol=tol, atol=tol)


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
@pytest.mark.parametrize("k,d,n", [(3, 5, 50001), (4, 6, 127), (8, 8, 9000)])
def test_fcm_small_no_labels(gpu, dt, k, d, n):
    """The fit's step form (labels = None) == with labels; labels == argmax membership."""
    from tensorflow_distributed_clustering_amd import _native
    ops = _native.require()
    g = torch.Generator().manual_seed(k * 11 + n)
    x = torch.randn(n, d, generator=g, dtype=torch.float64).to(dt).to(gpu)
    c = torch.randn(k, d, generator=g, dtype=torch.float64).to(dt).to(gpu)
    out = []
    for lab in (torch.full((n,), -1, dtype=torch.int32, device=gpu), None):
        wx = torch.zeros(k, d, dtype=torch.float64, device=gpu)
        ws = torch.zeros(k, dtype=torch.float64, device=gpu)
        ops.fcm_small(x, c, 5.0, True, lab, wx, ws)
        out.append((wx, ws, lab))
    u = ref.fcm_memberships(x.double(), c.double(), 5.0, True)
    agree = (u.argmax(1).to(torch.int32) == out[0][2]).float().mean().item()
    assert agree > 0.999, agree
    tol = 1e-10 if dt == torch.float64 else 1e-5
    torch.testing.assert_close(out[1][0], out[0][0], rtol=tol, atol=tol)
    torch.testing.assert_close(out[1][1], out[0][1], rtol=tol, atol=tol)


@pytest.mark.parametrize("m", [2.0, 3.0])
def test_fcm_mfma_blobs_accuracy(gpu, m):
    """The register tower on clustered data (Gaussian blobs, centroids next to blob rows):
    one-product stats pass with the two-nearest fix-up and bf16 weights in W^T X stay at the
    accuracy the bf16x3 distances set (profiles/fcm_bf16_w_ab_r04u.txt: 1.1e-3 of max|c| at
    m=2, 5.5e-3 at m=3 against the fp64 oracle)."""
    from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
    from tensorflow_distributed_clustering_amd.ops import HipMfmaFCM
    g = torch.Generator().manual_seed(0)
    x = gaussian_blobs(100_000, 128, 1024, seed=3, dtype=torch.float64, device="cpu")
    c = x[torch.randperm(x.shape[0], generator=g)[:1024]] + 0.1
    xg, cg = x.float().to(gpu), c.float().to(gpu)
    ops = HipMfmaFCM(xg, 1024, m, True)
    lab = torch.empty(x.shape[0], dtype=torch.int32, device=gpu)
    wx = torch.zeros(1024, 128, dtype=torch.float64, device=gpu)
    ws = torch.zeros(1024, dtype=torch.float64, device=gpu)
    ops.step(cg, lab, wx, ws)
    # fp64 exact-difference oracle, on the GPU (row chunks)
    a, b, lr = ref.fcm_partial(xg.double(), cg.double(), m, True, exact=True)
    a, b, lr = a.cpu(), b.cpu(), lr.cpu()
    cen = (wx / ws.clamp_min(1e-300)[:, None]).cpu()
    cref = a / b.clamp_min(1e-300)[:, None]
    ok = b > 1e-6 * b.max()
    err = float((cen[ok] - cref[ok]).abs().max() / cref[ok].abs().max())
    assert err < (3e-3 if m == 2.0 else 1.2e-2), err
    # weight sums: a few percent on the smallest-sum centroids at m = 3 (the same with the W
    # hi/lo split: profiles/fcm_bf16_w_ab_r04u.txt)
    torch.testing.assert_close(ws.cpu()[ok], b[ok], rtol=1e-2 if m == 2.0 else 4e-2,
                               atol=1e-6 * float(b.max()))
    assert (lab.long().cpu() == lr.long()).double().mean().item() > 0.999


@pytest.mark.parametrize("k,d", [(1024, 128), (257, 64)])
@pytest.mark.parametrize("m", [2.0, 1.5])
@pytest.mark.parametrize("nz", [True, False])
def test_fcm_mfma_one_product_vs_bf16x3(gpu, k, d, m, nz):
    """From D = 64 the accumulate pass runs one-product distances with the stats pass's
    two-nearest fix-up (HipMfmaFCM.one_product); the bf16x3 form (one_product = False)
    on the same data and centroids must agree with it to well inside the oracle
    tolerance, and both must meet the oracle, and the precision string must say which."""
    from tensorflow_distributed_clustering_amd.ops import FCM_PRECISION, HipMfmaFCM
    n = 20001
    x, c = _data(n, k, d, 11 * k + d)
    xg, cg = x.float().to(gpu), c.float().to(gpu)
    res = {}
    for one in (True, False):
        ops = HipMfmaFCM(xg, k, m, nz)
        ops.one_product = one
        lab = torch.empty(n, dtype=torch.int32, device=gpu)
        wx = torch.zeros(k, d, dtype=torch.float64, device=gpu)
        ws = torch.zeros(k, dtype=torch.float64, device=gpu)
        ops.step(cg, lab, wx, ws)
        assert ops.precision == FCM_PRECISION["bf16_one" if one else "bf16"]  # fp32 rows
        _check(wx.cpu(), ws.cpu(), lab, xg.cpu(), cg.cpu(), m, nz, 2e-3 * m, 0.998)
        res[one] = (wx.cpu(), ws.cpu(), lab.cpu())
    (wx1, ws1, l1), (wx3, ws3, l3) = res[True], res[False]
    ok = ws3 > 1e-12 * ws3.max()
    # a cluster whose sum is one dominant weight (the point that generated it) moves by
    # the bf16 rounding of that weight when its d2 moves by an fp32 ulp between the two
    # forms: up to 2^-8 each way, so two bf16 ulps
    assert float(((ws1 - ws3).abs() / ws3.clamp_min(1e-300))[ok].max()) < 2.0 ** -7
    c1, c3 = wx1 / ws1.clamp_min(1e-300)[:, None], wx3 / ws3.clamp_min(1e-300)[:, None]
    # and the two forms agree with each other at the oracle tolerance of _check
    tol = 2e-3 * m
    assert bool(((c1 - c3).abs() <= tol * (1 + c3.abs()))[ok].all())
    assert (l1 == l3).double().mean().item() >= 0.999


@pytest.mark.parametrize("k,d", [(1024, 128), (300, 100), (257, 64)])
@pytest.mark.parametrize("m", [2.0, 3.0])
@pytest.mark.parametrize("nz", [True, False])
def test_fcm_mfma_bf16_rows_raw_wtx(gpu, k, d, m, nz):
    """A bf16 shard: the accumulate pass takes the rows themselves as its one W^T X operand
    (exact bf16 products, no shift), padded when D < DP.  Against the fp64 oracle ON THE
    bf16 ROWS with the tower's tolerances, and against the hi/lo form (raw_rows = False)."""
    from tensorflow_distributed_clustering_amd.ops import FCM_PRECISION, HipMfmaFCM
    n = 20001
    x, c = _data(n, k, d, 13 * k + d)
    xb = x.to(torch.bfloat16)
    x[7] = xb[7].double()
    c[min(3, k - 1)] = xb[7].double()  # the on-centroid point, exactly, after the rounding
    xg, cg = xb.to(gpu), c.float().to(gpu)
    res = {}
    for raw in (True, False):
        ops = HipMfmaFCM(xg, k, m, nz)
        ops.one_product = True
        ops.raw_rows = raw
        lab = torch.empty(n, dtype=torch.int32, device=gpu)
        wx = torch.zeros(k, d, dtype=torch.float64, device=gpu)
        ws = torch.zeros(k, dtype=torch.float64, device=gpu)
        ops.step(cg, lab, wx, ws)
        assert (ops.xr is not None) == raw
        assert ops.precision == FCM_PRECISION["bf16_one_raw" if raw else "bf16_one"]
        # one-product distances of the far centroids (~2^-9 / sqrt(D) of |x||c|) on top of
        # the bf16 weights: this seed's worst cluster sum is 0.44 % off at m = 2 (the
        # bf16x3 tolerance of the fp32-row tests is 0.4 %)
        _check(wx.cpu(), ws.cpu(), lab, xb.double(), cg.cpu(), m, nz, 3e-3 * m, 0.998)
        res[raw] = (wx.cpu(), ws.cpu())
    (wx1, ws1), (wx2, ws2) = res[True], res[False]
    ok = ws2 > 1e-12 * ws2.max()
    c1, c2 = wx1 / ws1.clamp_min(1e-300)[:, None], wx2 / ws2.clamp_min(1e-300)[:, None]
    # same weights, same rows (hi + lo of the shifted bf16 rows sum back to them): only the
    # fp32 accumulation order differs
    torch.testing.assert_close(ws1, ws2, rtol=1e-6, atol=0)
    assert bool(((c1 - c2).abs() <= 1e-5 * (1 + c2.abs()))[ok].all())


def test_fcm_distances_config_selects_form(gpu):
    """ClusterConfig.fcm_distances reaches the MFMA tower: 'x3' runs the bf16x3 accumulate
    (precision string and engine attribute), 'one' the one-product form; both fits stay
    within the MFMA tower's tolerance of each other."""
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
    from tensorflow_distributed_clustering_amd.ops import FCM_PRECISION
    x = gaussian_blobs(30000, 128, 64, seed=3, dtype=torch.float32, device=gpu)
    cen = {}
    for mode in ("one", "x3"):
        cfg = tdc.ClusterConfig(n_clusters=64, max_iter=3, dtype="bf16", fuzzifier=2.0, seed=2,
                                fcm_distances=mode)
        f = tdc.FuzzyCMeans(cfg).fit(x)
        loc = f.engine_.local
        assert loc.one_product == (mode == "one")
        assert loc.precision == FCM_PRECISION["bf16_one" if mode == "one" else "bf16"]  # fp32
        cen[mode] = torch.as_tensor(f.result_.centers, dtype=torch.float64)
    # the one-product form moves the centroid of a fuzzy cluster: after 3 iterations on
    # this data by up to 1.5 % of max|c| (the rest agree to ~1e-5), the size of the
    # at-init witness gap of the fcm10m bench (9.4e-3 vs 9.0e-4)
    diff = (cen["one"] - cen["x3"]).abs().max(1).values
    assert float(diff.max()) < 3e-2 * float(cen["x3"].abs().max())
    assert float(diff.median()) < 1e-3 * float(cen["x3"].abs().max())


@pytest.mark.parametrize("k,d", [(1024, 128), (300, 100)])
@pytest.mark.parametrize("nz", [True, False])
def test_fcm_mfma_bf16x3_raw_wtx(gpu, k, d, nz):
    """bf16x3 distances (the default form) on a bf16 shard: the tile holds xh | xl | xr and
    W^T X takes the raw rows (one product); against the hi/lo W^T X of the same form the
    weights are identical and the centroids agree to the split's 2^-17."""
    from tensorflow_distributed_clustering_amd.ops import FCM_PRECISION, HipMfmaFCM
    n, m = 20001, 2.0
    x, c = _data(n, k, d, 17 * k + d)
    xb = x.to(torch.bfloat16)
    c[min(3, k - 1)] = xb[7].double()
    xg, cg = xb.to(gpu), c.float().to(gpu)
    res = {}
    for raw in (True, False):
        ops = HipMfmaFCM(xg, k, m, nz)
        ops.raw_rows = raw
        lab = torch.empty(n, dtype=torch.int32, device=gpu)
        wx = torch.zeros(k, d, dtype=torch.float64, device=gpu)
        ws = torch.zeros(k, dtype=torch.float64, device=gpu)
        ops.step(cg, lab, wx, ws)
        assert ops.precision == FCM_PRECISION["bf16_raw" if raw else "bf16"]
        # (the stats pass's one-product normaliser on bf16-rounded rows: this seed's worst
        # cluster sum is 0.41 % off at m = 2 in both W^T X forms)
        _check(wx.cpu(), ws.cpu(), lab, xb.double(), cg.cpu(), m, nz, 3e-3 * m, 0.998)
        res[raw] = (wx.cpu(), ws.cpu())
    (wx1, ws1), (wx2, ws2) = res[True], res[False]
    ok = ws2 > 1e-12 * ws2.max()
    torch.testing.assert_close(ws1, ws2, rtol=1e-6, atol=0)
    c1, c2 = wx1 / ws1.clamp_min(1e-300)[:, None], wx2 / ws2.clamp_min(1e-300)[:, None]
    assert bool(((c1 - c2).abs() <= 1e-5 * (1 + c2.abs()))[ok].all())



@pytest.mark.parametrize("k,d", [(1024, 128), (130, 100), (300, 17), (64, 256), (40, 768)])
@pytest.mark.parametrize("m", [2.0, 3.0, 5.0])
@pytest.mark.parametrize("nz", [True, False])
def test_fcm_f64_fused_matches_oracle(gpu, k, d, m, nz):
    """fp64 wide path with the row statistics fused into the f64-MFMA distance pass
    (fcm_f64t: t into G + rowinfo + labels, then W^T X with w formed while staging), over
    several chunks with a ragged tail and a point exactly on a centroid: the fp64 oracle's
    numbers, and the same labels / sums as the unfused three-kernel path."""
    from tensorflow_distributed_clustering_amd.ops import HipWideFCM
    n = 5003
    x, c = _data(n, k, d, 11 * k + d)
    xg, cg = x.to(gpu), c.to(gpu)
    res = {}
    for fused in (True, False):
        ops = HipWideFCM(xg, k, "fp64", m, nz)
        ops.fused = fused
        ops.chunk_elems = 2000 * k  # 3 chunks, the last ragged
        lab = torch.empty(n, dtype=torch.int32, device=gpu)
        wx = torch.zeros(k, d, dtype=torch.float64, device=gpu)
        ws = torch.zeros(k, dtype=torch.float64, device=gpu)
        ops.step(cg, lab, wx, ws)
        _check(wx.cpu(), ws.cpu(), lab, xg.cpu(), cg.cpu(), m, nz, 1e-9, 0.99999)
        lab2 = torch.full_like(lab, -1)
        ops.assign(cg, lab2)
        assert torch.equal(lab, lab2)
        res[fused] = (lab.cpu(), wx.cpu(), ws.cpu())
    assert torch.equal(res[True][0], res[False][0])
    torch.testing.assert_close(res[True][2], res[False][2], rtol=1e-11, atol=0)
