"""fp32 / fp64 K-Means assignment on the matrix cores (csrc/assign_x3.hip, ops.HipX3Lloyd).

The contract: labels equal the exact difference-form argmin in the data's own dtype, up to
that dtype's rounding of the distances (a row may differ only where two exact distances
tie within 1e-6 relative in fp32, 1e-12 in fp64).  The oracle is a plain PyTorch fp64
difference-form argmin; the fp32 comparison is also made against the native exact SIMT
tiles (assign_exact), the path the MFMA one replaces.
"""
import pytest
import torch

from tensorflow_distributed_clustering_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _blobs(n, d, k, seed, spread=3.0, dtype=torch.float64):
    g = torch.Generator(device="cpu").manual_seed(seed)
    c = torch.randn(k, d, generator=g, dtype=torch.float64) * spread
    lab = torch.randint(0, k, (n,), generator=g)
    x = c[lab] + torch.randn(n, d, generator=g, dtype=torch.float64)
    return x.to(dtype), c.to(dtype)


def _tie_ok(x64, c64, labels, rel):
    """Every label at the exact minimum, or within ``rel`` (relative) of it."""
    d = ref.pairwise_sqdist(x64, c64, exact=True)
    best, _ = d.min(1)
    got = d.gather(1, labels.long().cpu()[:, None]).squeeze(1)
    bad = got - best > rel * best.abs() + 1e-30
    return int(bad.sum()), best


def _x3(x, k, dtype):
    from tensorflow_distributed_clustering_amd.ops import HipX3Lloyd
    return HipX3Lloyd(x, k, dtype)


def _eps_rows(lo, n):
    """The kernel's per-row bound (assign_x3.hip x3_eps), recomputed on the host."""
    import math
    hx = lo.xh[:n].double().pow(2).sum(1).sqrt().cpu() * 1.0001
    lx = lo.xl[:n].double().pow(2).sum(1).sqrt().cpu() * 1.0001
    cn, h2, l2 = (float(v) for v in lo.cstat.cpu())
    Hc, Lc = math.sqrt(h2) * 1.0001, math.sqrt(l2) * 1.0001
    R8 = 2 ** -8 / (1 - 2 ** -8)
    KS = lo.dp // 32
    Rc, Rx = R8 * Lc, R8 * lx
    e_split = hx * Rc + lx * Lc + lx * Rc + Rx * Hc + Rx * Lc + Rx * Rc
    s_main, s_cross = hx * Hc, hx * Lc + lx * Hc
    U8 = 8 * 2 ** -23
    e_acc = U8 * (KS * cn + (KS + 1) * s_main) + U8 * (2 * KS + 1) * s_cross + \
        2 ** -24 * (cn + s_main + s_cross)
    return ((e_split + e_acc + 2 ** -23 * cn + 2 ** -19 * (cn + s_main + s_cross)) * 1.001).numpy()


@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
@pytest.mark.parametrize("n,d,k", [(20000, 20, 64), (30000, 64, 100), (50000, 128, 1024),
                                   (7777, 100, 257), (9000, 200, 130), (6000, 256, 64),
                                   (4000, 300, 70), (3000, 768, 1024), (2500, 1000, 40),
                                   (777, 128, 7)])
def test_x3_labels_exact(gpu, dtype, n, d, k):
    tdt = torch.float32 if dtype == "fp32" else torch.float64
    x, c = _blobs(n, d, k, seed=n + d + k, dtype=tdt)
    xg, C = x.to(gpu), c.to(gpu).contiguous()
    lo = _x3(xg, k, dtype)
    assert lo.name == "hip_x3_mfma"
    lo.prepare(C)
    labels = torch.full((n,), -1, dtype=torch.int32, device=gpu)
    lo.assign(C, labels, None)
    torch.cuda.synchronize()
    assert int(labels.min()) >= 0 and int(labels.max()) < k
    # fp32: the re-check's own difference-form rounding (positive terms, ~sqrt(D) 2^-24)
    rel = (1e-6 if d <= 256 else 4e-6) if dtype == "fp32" else 1e-12
    bad, _ = _tie_ok(x.double(), c.double(), labels, rel)
    assert bad == 0, f"{bad} rows off the exact argmin"
    # the ambiguous list stays small on blob data
    assert lo.ambiguous_rows() <= 0.2 * n


@pytest.mark.parametrize("n,d,k", [(40000, 128, 1024), (9000, 64, 300), (3000, 512, 256)])
def test_x3_matches_simt_exact_fp32(gpu, n, d, k):
    """fp32 labels of the MFMA path vs the native exact tiles (assign_exact)."""
    from tensorflow_distributed_clustering_amd import _native
    ops = _native.require()
    x, c = _blobs(n, d, k, seed=7 + d, dtype=torch.float32)
    xg, C = x.to(gpu), c.to(gpu).contiguous()
    lo = _x3(xg, k, "fp32")
    lo.prepare(C)
    la = torch.empty(n, dtype=torch.int32, device=gpu)
    lo.assign(C, la, None)
    lb = torch.empty(n, dtype=torch.int32, device=gpu)
    ops.assign_exact(xg, C, lb, None)
    diff = (la != lb).nonzero().flatten().cpu()
    if diff.numel():
        d64 = ref.pairwise_sqdist(x[diff].double(), c.double(), exact=True)
        da = d64.gather(1, la.cpu()[diff].long()[:, None]).squeeze(1)
        db = d64.gather(1, lb.cpu()[diff].long()[:, None]).squeeze(1)
        assert torch.all((da - db).abs() <= 1e-6 * db.abs() + 1e-30), "labels differ off a tie"


def test_x3_score_bound_holds(gpu):
    """The kernel's min distance (score of the winner + ||x||^2) is within the documented
    bound of the exact distance of its label (no re-check: raw MFMA scores)."""
    from tensorflow_distributed_clustering_amd import _native
    ops = _native.require()
    n, d, k = 20000, 128, 512
    x, c = _blobs(n, d, k, seed=11, spread=10.0, dtype=torch.float32)
    xg, C = x.to(gpu), c.to(gpu).contiguous()
    lo = _x3(xg, k, "fp32")
    lo.prepare(C)
    labels = torch.empty(n, dtype=torch.int32, device=gpu)
    mind = torch.empty(n, dtype=torch.float32, device=gpu)
    ops.x3_assign(lo.x, lo.xh[:n], lo.xl[:n], lo.ch, lo.cl, lo.cnorm, lo.cnhl, C, labels, mind,
                  lo.amb[: 3 * n], lo.cstat, lo.amb_count, False)
    torch.cuda.synchronize()
    x64, c64 = x.double(), c.double()
    exact = ((x64 - c64[labels.long().cpu()]) ** 2).sum(1)
    eps = torch.as_tensor(_eps_rows(lo, n), dtype=torch.float64)
    # mind = score + fp32 ||xh + xl||^2 of the split row: allow that sum's own rounding
    xn = (x64 * x64).sum(1)
    err = (mind.double().cpu() - exact).abs()
    slack = 2 ** -14 * xn
    assert torch.all(err <= eps + slack), float(((err - slack) / eps).max())
    # the bound is not vacuous: the observed score error is a small part of it
    assert float(((err - slack).clamp_min(0) / eps).max()) < 0.5


def test_x3_duplicate_centroids_full_scan(gpu):
    """Three identical centroids: the rows near them have no certifiable top-2 and take
    the full exact scan; ties resolve to the lowest index, as the exact argmin."""
    n, d, k = 6000, 96, 40
    x, c = _blobs(n, d, k, seed=3, dtype=torch.float32)
    c[9] = c[4]
    c[17] = c[4]
    c[30] = c[12]
    xg, C = x.to(gpu), c.to(gpu).contiguous()
    lo = _x3(xg, k, "fp32")
    lo.prepare(C)
    labels = torch.empty(n, dtype=torch.int32, device=gpu)
    lo.assign(C, labels, None)
    lab = labels.cpu()
    assert not bool(((lab == 9) | (lab == 17) | (lab == 30)).any())
    bad, _ = _tie_ok(x.double(), c.double(), labels, 1e-6)
    assert bad == 0


def test_x3_near_ties_fp64(gpu):
    """Rows placed (almost) halfway between two centroids: labels are the fp64 argmin."""
    g = torch.Generator().manual_seed(5)
    n, d, k = 8192, 128, 64
    c = torch.randn(k, d, generator=g, dtype=torch.float64) * 4
    a = torch.randint(0, k, (n,), generator=g)
    b = (a + 1 + torch.randint(0, k - 1, (n,), generator=g)) % k
    t = 0.5 + (torch.rand(n, generator=g, dtype=torch.float64) - 0.5) * 1e-6
    x = c[a] * t[:, None] + c[b] * (1 - t[:, None])
    xg, C = x.to(gpu), c.to(gpu).contiguous()
    lo = _x3(xg, k, "fp64")
    lo.prepare(C)
    labels = torch.empty(n, dtype=torch.int32, device=gpu)
    lo.assign(C, labels, None)
    bad, _ = _tie_ok(x, c, labels, 1e-12)
    assert bad == 0
    assert lo.ambiguous_rows() > n // 2  # the bound flags the near ties


@pytest.mark.parametrize("d", [64, 128, 768])
def test_kmeans_fit_fp32_mfma_vs_simt(gpu, d):
    """End to end: fp32 K-Means on the MFMA path and on the SIMT exact tiles."""
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
    n, k = 60000 if d < 768 else 12000, 256
    x = gaussian_blobs(n, d, k, seed=2, dtype=torch.float32, device=gpu)
    cfg = tdc.ClusterConfig(n_clusters=k, dtype="fp32", max_iter=8, seed=1)
    a = tdc.KMeans(cfg).fit(x)
    b = tdc.KMeans(cfg.replace(exact_assign="simt")).fit(x)
    assert a.result_.backend == "hip_x3_mfma" and b.result_.backend != "hip_x3_mfma"
    agree = float((a.result_.labels == b.result_.labels).double().mean())
    assert agree >= 0.9999
    import numpy as np
    np.testing.assert_allclose(a.result_.centers, b.result_.centers, rtol=1e-4, atol=1e-4)


def test_x3_streamed_and_delta(gpu):
    """Streamed chunks (bind re-splits each chunk) and the delta update on the x3 ops."""
    import numpy as np
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
    n, d, k = 50000, 128, 128
    x = gaussian_blobs(n, d, k, seed=4, dtype=torch.float32, device="cpu")
    cfg = tdc.ClusterConfig(n_clusters=k, dtype="fp32", max_iter=6, seed=3)
    res = tdc.KMeans(cfg).fit(x.to(gpu)).result_
    st = tdc.KMeans(cfg.replace(chunk_rows=12345), device=gpu).fit(x).result_
    assert st.streamed and st.backend == "hip_x3_mfma"
    np.testing.assert_allclose(res.centers, st.centers, rtol=1e-5, atol=1e-5)
    full = tdc.KMeans(cfg.replace(update="full")).fit(x.to(gpu)).result_
    np.testing.assert_allclose(res.centers, full.centers, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("n,m", [(60000, 1), (60000, 100), (60000, 700), (60000, 1700),
                                 (60000, 40000), (20000, 100), (20000, 700), (20000, 5000)])
def test_listed_rescan_matches_exact(gpu, dtype, n, m):
    """The listed full re-scan (x3_recheck's listF part): short lists run on the few-rows
    kernel (<= 32768 rows; 2 / 4 / 8 rows per workgroup by the listed count: m = 100 / 700 /
    1700+), long ones on the 128-row tiles; the K-split merge runs in the tiled launch
    (n > 32768) or in its own kernel (n = 20000).  All give the labels of the full exact
    tiles on the listed rows and leave the other rows alone."""
    from tensorflow_distributed_clustering_amd import _native
    ops = _native.require()
    d, k = 100, 700  # three 256-centroid chunks: K splits of 1 to 3
    x, c = _blobs(n, d, k, seed=m, dtype=dtype)
    xg, C = x.to(gpu), c.to(gpu).contiguous()
    want = torch.empty(n, dtype=torch.int32, device=gpu)
    ops.assign_exact(xg, C, want, None)
    rows = torch.randperm(n, generator=torch.Generator().manual_seed(m))[:m].to(torch.int32)
    cap = n
    amb = torch.zeros(3 * cap, dtype=torch.int32, device=gpu)
    amb[2 * cap: 2 * cap + m] = rows.to(gpu)
    count = torch.tensor([0, m], dtype=torch.int32, device=gpu)
    labels = torch.full((n,), -1, dtype=torch.int32, device=gpu)
    ops.x3_recheck(xg, C, labels, amb, count)
    torch.cuda.synchronize()
    got = labels.cpu()
    listed = torch.zeros(n, dtype=torch.bool)
    listed[rows.long()] = True
    assert torch.equal(got[listed], want.cpu()[listed])
    assert bool((got[~listed] == -1).all())


@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
@pytest.mark.parametrize("n,d,k,offset", [(50000, 128, 1024, 0.0), (30000, 64, 200, 0.0),
                                          (6000, 256, 64, 0.0), (40000, 128, 256, 200.0)])
def test_x3_prefilter_same_labels(gpu, dtype, n, d, k, offset):
    """The one-product prefilter only decides rows its own bound certifies: the labels are
    those of the plain three-product pass (both exact up to the dtype's rounding).  The
    offset case (|x| >> the cluster gaps): the split subtracts a fixed shift (the rows'
    mean), so the bounds scale with the spread and the offset data certifies as well as
    centred data (before the shift it left most rows to the three products and the exact
    re-scan)."""
    tdt = torch.float32 if dtype == "fp32" else torch.float64
    x, c = _blobs(n, d, k, seed=d + k, dtype=tdt)
    x, c = x + offset, c + offset
    xg, C = x.to(gpu), c.to(gpu).contiguous()
    lo = _x3(xg, k, dtype)
    assert lo.pre is not None and lo.prefilter
    lo.prepare(C)
    la = torch.full((n,), -1, dtype=torch.int32, device=gpu)
    lo.assign(C, la, None)
    listed = lo.prefilter_rows()
    lo.prefilter = False
    lb = torch.full((n,), -1, dtype=torch.int32, device=gpu)
    lo.assign(C, lb, None)
    assert lo.prefilter_rows() == 0
    rel = 1e-6 if dtype == "fp32" else 1e-12
    bad, _ = _tie_ok(x.double(), c.double(), la, rel)
    assert bad == 0
    diff = (la != lb).nonzero().flatten().cpu()
    if diff.numel():  # only exact ties may differ
        d64 = ref.pairwise_sqdist(x[diff].double(), c.double(), exact=True)
        da = d64.gather(1, la.cpu()[diff].long()[:, None]).squeeze(1)
        db = d64.gather(1, lb.cpu()[diff].long()[:, None]).squeeze(1)
        assert torch.all((da - db).abs() <= rel * db.abs() + 1e-30)
    assert listed < 0.5 * n, listed  # blob data: most rows certify on one product
    assert lo.ambiguous_rows() <= 0.2 * n  # ... and on three


def _near_ties(n, d, k, seed, dtype, delta=1e-3):
    """Rows between two random centroids at t = 0.5 +- delta: a distance gap of ~4 delta
    ||c_a - c_b||^2, below the one-product bound (~2^-8 |x||c|) and far above the
    three-product one, at any shift."""
    g = torch.Generator().manual_seed(seed)
    c = torch.randn(k, d, generator=g, dtype=torch.float64) * 4
    a = torch.randint(0, k, (n,), generator=g)
    b = (a + 1 + torch.randint(0, k - 1, (n,), generator=g)) % k
    t = 0.5 + (torch.rand(n, generator=g, dtype=torch.float64) - 0.5) * 2 * delta
    x = c[a] * t[:, None] + c[b] * (1 - t[:, None])
    return x.to(dtype), c.to(dtype)


def test_x3_prefilter_backs_off(gpu):
    """Data where the one-product bound certifies almost nothing (rows near ties of two
    centroids): once the listed count has come back, the prefilter is skipped for
    PRE_RETRY assignments, and the labels stay exact either way."""
    n, d, k = 20000, 128, 128
    x, c = _near_ties(n, d, k, seed=9, dtype=torch.float32)
    xg, C = x.to(gpu), c.to(gpu).contiguous()
    lo = _x3(xg, k, "fp32")
    lo.prepare(C)
    labels = torch.empty(n, dtype=torch.int32, device=gpu)
    lo.assign(C, labels, None)
    assert lo.prefilter_rows() > lo.PRE_MAX_FRAC * n
    torch.cuda.synchronize()
    lo.assign(C, labels, None)
    assert lo.prefilter_rows() == 0  # skipped: the first count was read
    for _ in range(lo.PRE_RETRY - 1):
        lo.assign(C, labels, None)
    assert lo.prefilter_rows() == 0
    lo.assign(C, labels, None)
    assert lo.prefilter_rows() > 0  # tried again after PRE_RETRY skipped assignments
    bad, _ = _tie_ok(x.double(), c.double(), labels, 1e-6)
    assert bad == 0


@pytest.mark.parametrize("frac", [0.0, 1.0])
def test_x3_listed_launch_estimate(gpu, frac):
    """The listed bf16x3 launch is sized from the previous listed share: a low estimate
    leaves the rest to the grid-stride overflow launch, a high one to workgroups that
    leave at once; the labels are exact either way."""
    n, d, k = 60000, 128, 128
    x, c = _near_ties(n, d, k, seed=21, dtype=torch.float32)  # almost every row listed
    xg, C = x.to(gpu), c.to(gpu).contiguous()
    lo = _x3(xg, k, "fp32")
    lo.prepare(C)
    lo.PRE_MAX_FRAC = 2.0  # never back off here
    lo._pre_frac = frac
    labels = torch.full((n,), -1, dtype=torch.int32, device=gpu)
    lo.assign(C, labels, None)
    assert lo.prefilter_rows() > 40000
    bad, _ = _tie_ok(x.double(), c.double(), labels, 1e-6)
    assert bad == 0


def test_x3_listed_overflow_multiblock(gpu):
    """The listed launch's grid-stride overflow kernel (LISTED = 2) with several point
    blocks per workgroup: the LDS ring is reused across blocks (the __syncthreads before
    each later block) and the lane constants are rebuilt per block.  ~1M listed rows against
    a one-shot launch sized for 16K (the estimate of a share of 0) leave the overflow grid
    (<= the resident workgroups, 256 rows each) >= 3 blocks per workgroup; the labels are
    the fp64 argmin."""
    from tensorflow_distributed_clustering_amd import _native
    n, d, k = 1_000_000, 128, 64
    x, c = _near_ties(n, d, k, seed=33, dtype=torch.float32)
    xg, C = x.to(gpu), c.to(gpu).contiguous()
    lo = _x3(xg, k, "fp32")
    lo.prepare(C)
    lo.PRE_MAX_FRAC = 2.0
    lo._pre_frac = 0.0
    labels = torch.full((n,), -1, dtype=torch.int32, device=gpu)
    lo.assign(C, labels, None)
    torch.cuda.synchronize()
    listed = lo.prefilter_rows()
    cus = torch.cuda.get_device_properties(gpu).multi_processor_count
    assert listed - 16384 > 3 * (4 * cus) * 256, (listed, cus)  # >= 3 blocks per workgroup
    assert int(labels.min()) >= 0
    bad, _ = _tie_ok(x.double(), c.double(), labels, 1e-6)
    assert bad == 0
