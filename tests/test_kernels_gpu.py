"""Numerics of every HIP kernel against a plain-PyTorch fp64 reference of the same op.

Label checks tolerate only *near ties*: a row may pick a different centroid than the
fp64 oracle only if that centroid's exact distance is within the kernel's arithmetic
error of the optimum.
"""
import pytest
import torch

from tensorflow_distributed_clustering_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _bf16_case(n, d, k, dev, seed=0, spread=3.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    c = torch.randn(k, d, generator=g, dtype=torch.float64) * spread
    lab = torch.randint(0, k, (n,), generator=g)
    x = c[lab] + torch.randn(n, d, generator=g, dtype=torch.float64)
    return x.to(torch.bfloat16).to(dev), c.to(dev)


def _check_labels(x64, c64, labels, rel=2e-5):
    d = ref.pairwise_sqdist(x64, c64, exact=True)
    best, _ = d.min(1)
    got = d.gather(1, labels.long()[:, None]).squeeze(1)
    scale = (x64 * x64).sum(1) + (c64 * c64).sum(1).max()
    bad = (got - best) > rel * scale + 1e-9
    assert int(bad.sum()) == 0, f"{int(bad.sum())} rows not at a (near-)minimum"
    return best


@pytest.mark.parametrize("n,d,k", [(1000, 5, 3), (4097, 32, 64), (12345, 64, 100),
                                   (30000, 128, 1024), (5000, 100, 257), (3000, 256, 130),
                                   (777, 128, 15)])
def test_assign_bf16_mfma(gpu, n, d, k):
    from tensorflow_distributed_clustering_amd.ops import HipBf16Lloyd
    xb, c = _bf16_case(n, d, k, gpu, seed=n + d + k)
    loc = HipBf16Lloyd(xb, k)
    C = c.float().contiguous()
    loc.prepare(C)
    labels = torch.full((n,), -1, dtype=torch.int32, device=gpu)
    mind = torch.zeros(n, dtype=torch.float32, device=gpu)
    loc.assign(C, labels, mind)
    torch.cuda.synchronize()
    assert int(labels.min()) >= 0 and int(labels.max()) < k
    x64 = xb.double()
    c64 = C.to(torch.bfloat16).double()  # the kernel sees bf16-rounded centroids
    best = _check_labels(x64, c64, labels)
    scale = (x64 * x64).sum(1) + (c64 * c64).sum(1).max()
    assert torch.all((mind.double() - best).abs() <= 5e-5 * scale + 1e-4)


def test_assign_bf16_exact_integers(gpu):
    """Small-integer data: every product and sum is exact -> labels must match exactly."""
    from tensorflow_distributed_clustering_amd.ops import HipBf16Lloyd
    g = torch.Generator().manual_seed(5)
    n, d, k = 2048, 128, 192
    x = torch.randint(-4, 5, (n, d), generator=g).to(torch.float64)
    c = torch.randint(-4, 5, (k, d), generator=g).to(torch.float64)
    c[7] = c[3]  # exact duplicate centroid: ties must resolve to the lower index
    loc = HipBf16Lloyd(x.to(torch.bfloat16).to(gpu), k)
    C = c.float().to(gpu).contiguous()
    loc.prepare(C)
    labels = torch.empty(n, dtype=torch.int32, device=gpu)
    mind = torch.empty(n, dtype=torch.float32, device=gpu)
    loc.assign(C, labels, mind)
    dref = ref.pairwise_sqdist(x, c, exact=True)
    vref, lref = dref.min(1)
    assert torch.equal(mind.double().cpu(), vref)
    # exact distances; with the 5-bit index embedding an exact tie may pick either
    # of the tied centroids but never a non-minimal one
    got = dref.gather(1, labels.long().cpu()[:, None]).squeeze(1)
    assert torch.equal(got, vref)
    # centroids 3 and 7 sit in different lane halves: the cross-half tie-break picks 3
    assert not bool((labels.cpu() == 7).any())


@pytest.mark.parametrize("xdt", [torch.bfloat16, torch.float32, torch.float64])
@pytest.mark.parametrize("n,d,k", [(10000, 5, 3), (20000, 128, 1024), (5000, 33, 70), (3000, 300, 40)])
def test_update_lds(gpu, xdt, n, d, k):
    from tensorflow_distributed_clustering_amd import _native
    ops = _native.require()
    g = torch.Generator().manual_seed(n + d)
    x = torch.randn(n, d, generator=g).to(xdt).to(gpu)
    lab = torch.randint(0, k, (n,), generator=g, dtype=torch.int32).to(gpu)
    lab[:7] = 0  # make sure a hot cluster exists
    for acc in (torch.float32, torch.float64):
        sums = torch.zeros(k, d, dtype=acc, device=gpu)
        counts = torch.zeros(k, dtype=acc, device=gpu)
        ops.update(x, lab, sums, counts)
        s_ref, c_ref = ref.cluster_sums(x.double(), lab, k, acc_dtype=torch.float64)
        assert torch.equal(counts.double(), c_ref)
        tol = 1e-3 if acc == torch.float32 or xdt != torch.float64 else 1e-9
        torch.testing.assert_close(sums.double(), s_ref, rtol=tol, atol=tol * 10)


@pytest.mark.parametrize("xdt", [torch.bfloat16, torch.float32, torch.float64])
@pytest.mark.parametrize("n,d,k", [(10000, 5, 3), (50000, 128, 1024), (5000, 33, 70),
                                   (3000, 300, 40), (20000, 64, 5000), (4000, 768, 20000),
                                   (300000, 16, 16384), (777, 8, 4)])
def test_update_sorted(gpu, xdt, n, d, k):
    from tensorflow_distributed_clustering_amd import _native
    ops = _native.require()
    g = torch.Generator().manual_seed(n + d + 1)
    x = torch.randn(n, d, generator=g).to(xdt).to(gpu)
    lab = torch.randint(0, k, (n,), generator=g, dtype=torch.int32).to(gpu)
    lab[: n // 3] = 1  # one long segment spanning many waves
    work = torch.zeros(int(ops.update_sorted_workspace(n, k)), dtype=torch.int32, device=gpu)
    s_ref, c_ref = ref.cluster_sums(x.double(), lab, k, acc_dtype=torch.float64)
    for acc in (torch.float32, torch.float64):
        sums = torch.zeros(k, d, dtype=acc, device=gpu)
        counts = torch.zeros(k, dtype=acc, device=gpu)
        ops.update_sorted(x, lab, sums, counts, work)
        ops.update_sorted(x, lab, sums, counts, work)  # accumulates (streamed chunks)
        assert torch.equal(counts.double(), 2 * c_ref)
        tol = 1e-3 if acc == torch.float32 or xdt != torch.float64 else 1e-9
        torch.testing.assert_close(sums.double(), 2 * s_ref, rtol=tol, atol=tol * 10)


@pytest.mark.parametrize("n,k", [(2_500_000, 1024), (1_250_000, 1024)])
def test_update_sorted_scatter_passes(gpu, n, k):
    """Large per-block label ranges (>= 8 labels per bin per block) scatter in two bin-range
    passes: the permutation in the workspace is still every row exactly once, grouped by
    label, and the sums / counts match the fp64 oracle (1.25M rows: the one-pass form)."""
    from tensorflow_distributed_clustering_amd import _native
    ops = _native.require()
    d = 128
    g = torch.Generator().manual_seed(n + 7)
    x = torch.randn(n, d, generator=g).to(torch.bfloat16).to(gpu)
    lab = torch.randint(0, k, (n,), generator=g, dtype=torch.int32).to(gpu)
    lab[: n // 5] = 3  # one hot bin
    work = torch.zeros(int(ops.update_sorted_workspace(n, k)), dtype=torch.int32, device=gpu)
    sums = torch.zeros(k, d, dtype=torch.float32, device=gpu)
    counts = torch.zeros(k, dtype=torch.float32, device=gpu)
    ops.update_sorted(x, lab, sums, counts, work)
    perm = work[3 * k + 1: 3 * k + 1 + n].long()
    assert torch.equal(torch.sort(perm).values, torch.arange(n, device=gpu))
    grouped = lab[perm]
    assert bool((grouped[1:] >= grouped[:-1]).all())
    s_ref, c_ref = ref.cluster_sums(x.double(), lab, k, acc_dtype=torch.float64)
    assert torch.equal(counts.double(), c_ref)
    torch.testing.assert_close(sums.double(), s_ref, rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("n,k", [(1_250_000, 1024), (40_000, 4096), (3000, 64)])
def test_update_sorted_zero_first_and_clean_workspace(gpu, n, k):
    """zero_first: the all-reduce buffer [sums | counts | tail] full of garbage is cleared by
    the update's first kernel before anything accumulates (the engine's step needs no fill
    launch); the workspace histogram is left zeroed for the next call."""
    from tensorflow_distributed_clustering_amd import _native
    ops = _native.require()
    d = 128
    g = torch.Generator().manual_seed(n + k)
    x = torch.randn(n, d, generator=g).to(torch.bfloat16).to(gpu)
    lab = torch.randint(0, k, (n,), generator=g, dtype=torch.int32).to(gpu)
    work = torch.zeros(int(ops.update_sorted_workspace(n, k)), dtype=torch.int32, device=gpu)
    buf = torch.full((k * d + k + 7,), 123.0, dtype=torch.float32, device=gpu)
    sums, counts = buf[: k * d].view(k, d), buf[k * d: k * d + k]
    ops.update_sorted(x, lab, sums, counts, work, None, None, buf)
    torch.cuda.synchronize()
    assert int(work[:k].abs().sum()) == 0
    s_ref, c_ref = ref.cluster_sums(x.double(), lab, k, acc_dtype=torch.float64)
    assert torch.equal(counts.double(), c_ref)
    assert torch.equal(buf[k * d + k:], torch.zeros(7, device=gpu))
    torch.testing.assert_close(sums.double(), s_ref, rtol=1e-3, atol=1e-2)


def test_update_sorted_large_zero_fill_small_rows_and_dirty_workspace(gpu):
    """A few rows next to a large all-reduce buffer (the fill gets blocks of its own, 16-B
    stores, ragged tail), and a workspace with a dirty histogram: work_clean=False (the
    default) clears it first, so the counts are still right."""
    from tensorflow_distributed_clustering_amd import _native
    ops = _native.require()
    n, k, d = 700, 4096, 256
    g = torch.Generator().manual_seed(17)
    x = torch.randn(n, d, generator=g).to(torch.bfloat16).to(gpu)
    lab = torch.randint(0, k, (n,), generator=g, dtype=torch.int32).to(gpu)
    work = torch.randint(1, 9, (int(ops.update_sorted_workspace(n, k)),), generator=g,
                         dtype=torch.int32).to(gpu)  # garbage histogram
    buf = torch.full((k * d + k + 4096 * 1024 + 3,), 5.0, dtype=torch.float32, device=gpu)
    sums, counts = buf[: k * d].view(k, d), buf[k * d: k * d + k]
    ops.update_sorted(x, lab, sums, counts, work, None, None, buf)
    torch.cuda.synchronize()
    s_ref, c_ref = ref.cluster_sums(x.double(), lab, k, acc_dtype=torch.float64)
    assert torch.equal(counts.double(), c_ref)
    assert float(buf[k * d + k:].abs().max()) == 0.0
    torch.testing.assert_close(sums.double(), s_ref, rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
@pytest.mark.parametrize("k,d", [(3, 5), (6, 5), (9, 5), (12, 5), (15, 5), (16, 5), (8, 2),
                                 (16, 8), (4, 16), (32, 3)])
def test_lloyd_small_fused(gpu, dt, k, d):
    from tensorflow_distributed_clustering_amd import _native
    ops = _native.require()
    if not ops.lloyd_small_supported(dt, k, d):
        pytest.skip("tile not compiled for this dtype")
    g = torch.Generator().manual_seed(k * 100 + d)
    n = 50000
    x = torch.randn(n, d, generator=g, dtype=torch.float64).to(dt).to(gpu)
    c = torch.randn(k, d, generator=g, dtype=torch.float64).to(dt).to(gpu)
    labels = torch.empty(n, dtype=torch.int32, device=gpu)
    mind = torch.empty(n, dtype=dt, device=gpu)
    sums = torch.zeros(k, d, dtype=torch.float64, device=gpu)
    counts = torch.zeros(k, dtype=torch.float64, device=gpu)
    ops.lloyd_small(x, c, labels, mind, sums, counts)
    x64, c64 = x.double(), c.double()
    lref, mref = ref.assign(x64, c64, exact=True)
    if dt == torch.float64:
        assert torch.equal(labels, lref)
    else:
        _check_labels(x64, c64, labels, rel=1e-6)
    s_ref, c_ref = ref.cluster_sums(x64, labels, k)
    assert torch.equal(counts, c_ref)
    tol = 1e-10 if dt == torch.float64 else 2e-4
    torch.testing.assert_close(sums, s_ref, rtol=tol, atol=tol)
    torch.testing.assert_close(mind.double(), mref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
@pytest.mark.parametrize("k,d,n", [(3, 5, 50001), (4, 6, 127), (8, 8, 9000)])
def test_lloyd_small_no_labels(gpu, dt, k, d, n):
    """The fit's step form (labels = None, the final label pass writes them) == with labels."""
    from tensorflow_distributed_clustering_amd import _native
    ops = _native.require()
    g = torch.Generator().manual_seed(k * 7 + n)
    x = torch.randn(n, d, generator=g, dtype=torch.float64).to(dt).to(gpu)
    c = torch.randn(k, d, generator=g, dtype=torch.float64).to(dt).to(gpu)
    out = []
    for lab in (torch.full((n,), -1, dtype=torch.int32, device=gpu), None):
        sums = torch.zeros(k, d, dtype=torch.float64, device=gpu)
        counts = torch.zeros(k, dtype=torch.float64, device=gpu)
        ops.lloyd_small(x, c, lab, None, sums, counts)
        out.append((sums, counts, lab))
    assert int(out[0][2].min()) >= 0
    s_ref, c_ref = ref.cluster_sums(x.double(), out[0][2], k)
    assert torch.equal(out[0][1], c_ref) and torch.equal(out[1][1], c_ref)
    tol = 1e-10 if dt == torch.float64 else 2e-4
    torch.testing.assert_close(out[1][0], s_ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
@pytest.mark.parametrize("k,d", [(300, 5), (1000, 17), (64, 32)])
def test_assign_simt(gpu, dt, k, d):
    from tensorflow_distributed_clustering_amd import _native
    ops = _native.require()
    g = torch.Generator().manual_seed(k + d)
    n = 20000
    x = torch.randn(n, d, generator=g, dtype=torch.float64).to(dt).to(gpu)
    c = torch.randn(k, d, generator=g, dtype=torch.float64).to(dt).to(gpu)
    labels = torch.empty(n, dtype=torch.int32, device=gpu)
    mind = torch.empty(n, dtype=dt, device=gpu)
    ops.assign_simt(x, c, labels, mind)
    lref, mref = ref.assign(x.double(), c.double(), exact=True)
    if dt == torch.float64:
        assert torch.equal(labels, lref)
    else:
        _check_labels(x.double(), c.double(), labels, rel=1e-6)
    torch.testing.assert_close(mind.double(), mref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
@pytest.mark.parametrize("k,d,m", [(3, 5, 5.0), (6, 5, 5.0), (9, 5, 5.0), (12, 5, 2.0),
                                   (15, 5, 5.0), (16, 5, 1.5), (24, 5, 5.0), (32, 5, 2.0),
                                   (48, 5, 5.0), (64, 5, 2.0),
                                   (3, 3, 2.0), (8, 2, 2.0),
                                   (6, 4, 1.7), (5, 3, 3.0), (4, 4, 4.0), (7, 2, 2.5)])
@pytest.mark.parametrize("nan_to_zero", [True, False])
def test_fcm_small(gpu, dt, k, d, m, nan_to_zero):
    from tensorflow_distributed_clustering_amd import _native
    ops = _native.require()
    if not ops.fcm_small_supported(dt, k, d):
        pytest.skip("tile not compiled")
    g = torch.Generator().manual_seed(k + d)
    n = 20000
    x = torch.randn(n, d, generator=g, dtype=torch.float64)
    c = torch.randn(k, d, generator=g, dtype=torch.float64)
    x[5] = c[1]  # a point exactly on a centroid exercises the NaN guard
    x, c = x.to(dt).to(gpu), c.to(dt).to(gpu)
    labels = torch.empty(n, dtype=torch.int32, device=gpu)
    wx = torch.zeros(k, d, dtype=torch.float64, device=gpu)
    ws = torch.zeros(k, dtype=torch.float64, device=gpu)
    ops.fcm_small(x, c, m, nan_to_zero, labels, wx, ws)
    a, b, lr = ref.fcm_partial(x.double(), c.double(), m, nan_to_zero)
    tol = 1e-9 if dt == torch.float64 else 2e-4
    torch.testing.assert_close(ws, b, rtol=tol, atol=tol)
    torch.testing.assert_close(wx, a, rtol=tol, atol=tol * 10)
    agree = (labels == lr).double().mean().item()
    assert agree > (0.9999 if dt == torch.float64 else 0.999)


@pytest.mark.parametrize("policy", ["keep", "nan", "zero"])
def test_finalize_and_prep(gpu, policy):
    from tensorflow_distributed_clustering_amd import _native
    from tensorflow_distributed_clustering_amd.ops import POLICY_CODES
    ops = _native.require()
    k, d = 70, 100
    g = torch.Generator().manual_seed(1)
    sums = torch.randn(k, d, generator=g, dtype=torch.float64).to(gpu)
    counts = torch.randint(0, 5, (k,), generator=g).double().to(gpu)
    counts[3] = 0
    C = torch.randn(k, d, generator=g).to(gpu)
    old = C.clone()
    shift = torch.zeros(1, device=gpu)
    cm2 = torch.zeros(128, 128, dtype=torch.bfloat16, device=gpu)
    cn = torch.zeros(128, device=gpu)
    ops.finalize(sums, counts, C, POLICY_CODES[policy], shift, cm2, cn)
    exp = ref.finalize(sums, counts, old, policy)
    torch.testing.assert_close(C, exp, equal_nan=True)
    cb = C.to(torch.bfloat16)
    torch.testing.assert_close(cm2[:k, :d], (-2 * cb.float()).to(torch.bfloat16), rtol=0, atol=0,
                               equal_nan=True)
    assert torch.all(cm2[:, d:] == 0) and torch.all(cm2[k:] == 0)
    assert torch.all(cn[k:] > 1e38)
    fin = torch.isfinite(C).all(1)
    torch.testing.assert_close(cn[:k][fin], (cb.float() ** 2).sum(1)[fin], rtol=1e-5, atol=1e-5)
    if policy == "keep":
        dd = ((C.double() - old.double()) ** 2).sum(1).max()
        torch.testing.assert_close(shift.double()[0], dd, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("xdt,ddt", [(torch.bfloat16, torch.float32), (torch.float32, torch.float32),
                                     (torch.float64, torch.float64), (torch.float32, torch.float64)])
@pytest.mark.parametrize("n,d,t", [(20000, 5, 8), (5000, 128, 10), (3001, 33, 1), (7000, 300, 12)])
def test_kpp_step(gpu, xdt, ddt, n, d, t):
    from tensorflow_distributed_clustering_amd import _native
    ops = _native.require()
    g = torch.Generator().manual_seed(n + d)
    x = torch.randn(n, d, generator=g).to(xdt).to(gpu)
    cand = torch.randn(t, d, generator=g, dtype=torch.float64).to(ddt).to(gpu)
    closest = (torch.rand(n, generator=g, dtype=torch.float64) * 2 * d).to(ddt).to(gpu)
    d2 = ((x.double()[None] - cand.double()[:, None]) ** 2).sum(-1)  # [t, n]
    pots = torch.zeros(16, dtype=torch.float64, device=gpu)
    ops.kpp_step(x, cand, closest, 0, pots)
    ref_pots = torch.minimum(d2, closest.double()[None]).sum(1)
    torch.testing.assert_close(pots[:t], ref_pots, rtol=1e-5, atol=1e-3)
    pots.zero_()
    c1 = closest.clone()
    ops.kpp_step(x, cand[:1].contiguous(), c1, 1, pots)
    ref_c = torch.minimum(d2[0], closest.double())
    torch.testing.assert_close(c1.double(), ref_c, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(pots[0], ref_c.sum(), rtol=1e-5, atol=1e-3)


def test_native_kmeanspp_matches_torch_path(gpu):
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
    from tensorflow_distributed_clustering_amd.models.init import init_kmeanspp
    from tensorflow_distributed_clustering_amd.parallel.dist import local_comm
    x = gaussian_blobs(50000, 8, 16, seed=1, dtype=torch.float64, device=gpu)
    comm = local_comm(gpu)
    native = init_kmeanspp(x, 0, 50000, 16, comm, 3)
    torch_path = init_kmeanspp(x.cpu(), 0, 50000, 16, local_comm(torch.device("cpu")), 3)
    torch.testing.assert_close(native.cpu(), torch_path, rtol=0, atol=0)


@pytest.mark.parametrize("n,b,d,k", [(50000, 20000, 128, 1024), (30000, 7777, 64, 4096),
                                     (20000, 5000, 256, 300)])
def test_indexed_assign_and_update(gpu, n, b, d, k):
    """Mini-batch kernels that read rows in place by index == the same kernels on the
    gathered batch (labels bitwise, counts exactly, sums to fp32 atomic-order tolerance)."""
    import tensorflow_distributed_clustering_amd.ops as ops_mod
    from tensorflow_distributed_clustering_amd import _native
    ops = _native.require()
    x, c = _bf16_case(n, d, k, gpu, seed=n + b)
    lo = ops_mod.make_lloyd_ops(x, k, "bf16", "hip")
    C = c.float().contiguous()
    lo.prepare(C)
    g = torch.Generator(device=gpu).manual_seed(7)
    idx = torch.randint(n, (b,), generator=g, device=gpu, dtype=torch.int32)
    lab_i = torch.full((b,), -1, dtype=torch.int32, device=gpu)
    md_i = torch.zeros(b, dtype=torch.float32, device=gpu)
    ops.assign_bf16_indexed(lo.x, idx, lo.cm2, lo.cnorm, lab_i, md_i)
    xb = lo.x.index_select(0, idx.long()).contiguous()
    lab_g = torch.full((b,), -1, dtype=torch.int32, device=gpu)
    md_g = torch.zeros(b, dtype=torch.float32, device=gpu)
    ops.assign_bf16(xb, lo.cm2, lo.cnorm, lab_g, md_g)
    assert torch.equal(lab_i, lab_g)
    assert torch.equal(md_i, md_g)
    work = torch.zeros(int(ops.update_sorted_workspace(b, k)), dtype=torch.int32, device=gpu)
    s_i = torch.zeros(k, d, dtype=torch.float32, device=gpu)
    c_i = torch.zeros(k, dtype=torch.float32, device=gpu)
    ops.update_sorted_indexed(lo.x, idx, lab_i, s_i, c_i, work)
    s_ref, c_ref = ref.cluster_sums(xb[:, :d].double(), lab_g, k, acc_dtype=torch.float64)
    assert torch.equal(c_i.double(), c_ref)
    torch.testing.assert_close(s_i.double(), s_ref, rtol=1e-4, atol=1e-3)
    # the mini-batch step's form: [sums | counts] buffer full of stale values, cleared by
    # the update's first kernel (zero_first) before anything accumulates into it
    buf = torch.full((k * d + k,), 7.0, dtype=torch.float32, device=gpu)
    s_z, c_z = buf[: k * d].view(k, d), buf[k * d:]
    ops.update_sorted_indexed(lo.x, idx, lab_i, s_z, c_z, work, None, None, True, buf)
    assert torch.equal(c_z.double(), c_ref)
    torch.testing.assert_close(s_z.double(), s_ref, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("d,k", [(128, 1024), (128, 64), (100, 300)])
def test_assign_large_shard_tiles(gpu, d, k):
    """Shards of >= 2^20 rows take the P=8 point-tile launch at D=128: labels and distances
    equal the indexed (P=4) kernel's bit for bit, and the tail rows are at the fp64
    oracle's (near-)minimum."""
    import tensorflow_distributed_clustering_amd.ops as ops_mod
    from tensorflow_distributed_clustering_amd import _native
    ops = _native.require()
    n = (1 << 20) + 12345
    x, c = _bf16_case(n, d, k, gpu, seed=d + k)
    lo = ops_mod.make_lloyd_ops(x, k, "bf16", "hip")
    C = c.float().contiguous()
    lo.prepare(C)
    lab = torch.full((n,), -1, dtype=torch.int32, device=gpu)
    md = torch.zeros(n, dtype=torch.float32, device=gpu)
    ops.assign_bf16(lo.x, lo.cm2, lo.cnorm, lab, md)
    idx = torch.arange(n, device=gpu, dtype=torch.int32)
    lab_i = torch.full((n,), -1, dtype=torch.int32, device=gpu)
    md_i = torch.zeros(n, dtype=torch.float32, device=gpu)
    ops.assign_bf16_indexed(lo.x, idx, lo.cm2, lo.cnorm, lab_i, md_i)
    assert torch.equal(lab, lab_i)
    assert torch.equal(md, md_i)
    sl = slice(n - 30000, n)
    _check_labels(x[sl].double(), C.to(torch.bfloat16).double(), lab[sl])


@pytest.mark.parametrize("cdt", [torch.float32, torch.float64])
def test_sculley_update(gpu, cdt):
    from tensorflow_distributed_clustering_amd import _native
    ops = _native.require()
    k, d, kp, dp = 300, 100, 320, 128
    g = torch.Generator().manual_seed(11)
    C = torch.randn(k, d, generator=g, dtype=torch.float64)
    v = torch.randint(0, 50, (k,), generator=g).double()
    cnt = torch.randint(0, 5, (k,), generator=g).float()
    sums = torch.randn(k, d, generator=g).float() * cnt[:, None]
    nv = v + cnt.double()
    upd = cnt > 0
    want = torch.where(upd[:, None], (v[:, None] * C.to(cdt).double() + sums.double())
                       / nv.clamp_min(1)[:, None], C.to(cdt).double())
    want_shift = ((want - C.to(cdt).double()) ** 2).sum(1).max()
    Cg, vg = C.to(cdt).to(gpu), v.to(gpu)
    shift = torch.zeros(1, dtype=torch.float32, device=gpu)
    cm2 = torch.full((kp, dp), 7.0, dtype=torch.bfloat16, device=gpu)
    cnorm = torch.zeros(kp, dtype=torch.float32, device=gpu)
    ops.sculley_update(sums.to(gpu), cnt.to(gpu), Cg, vg, shift, cm2, cnorm)
    tol = 1e-6 if cdt == torch.float32 else 1e-12
    torch.testing.assert_close(Cg.double().cpu(), want, rtol=tol, atol=tol)
    assert torch.equal(vg.cpu(), nv)
    assert abs(float(shift) - float(want_shift)) <= 1e-4 * float(want_shift)
    cb = Cg.float().to(torch.bfloat16).float()
    torch.testing.assert_close(cm2[:k, :d].float(), -2 * cb)
    assert (cm2[:k, d:] == 0).all() and (cm2[k:] == 0).all()
    torch.testing.assert_close(cnorm[:k], (cb * cb).sum(1), rtol=1e-5, atol=1e-4)
    assert (cnorm[k:] == 3e38).all()


@pytest.mark.parametrize("n,d,k", [(30000, 128, 1024), (20000, 64, 4096), (9000, 256, 200),
                                   (777, 128, 70)])
def test_assign_bf16_top2(gpu, n, d, k):
    """Top-2 epilogue: same labels as the plain kernel, d1 = its min distance, d2 = the
    second-smallest distance (fp64 oracle on the bf16 operands, bf16-level tolerance);
    the indexed form equals the gathered rows."""
    import tensorflow_distributed_clustering_amd.ops as ops_mod
    from tensorflow_distributed_clustering_amd import _native
    ops = _native.require()
    x, c = _bf16_case(n, d, k, gpu, seed=d + k)
    lo = ops_mod.make_lloyd_ops(x, k, "bf16", "hip")
    C = c.float().contiguous()
    lo.prepare(C)
    lab = torch.empty(n, dtype=torch.int32, device=gpu)
    d1 = torch.empty(n, dtype=torch.float32, device=gpu)
    d2 = torch.empty(n, dtype=torch.float32, device=gpu)
    ops.assign_bf16_top2(lo.x, None, lo.cm2, lo.cnorm, lab, d1, d2)
    lab0 = torch.empty_like(lab)
    md0 = torch.empty_like(d1)
    ops.assign_bf16(lo.x, lo.cm2, lo.cnorm, lab0, md0)
    assert torch.equal(lab, lab0)
    # equal up to the centroid-id bits embedded in the score mantissa (QT may differ)
    torch.testing.assert_close(d1, md0, rtol=1e-4, atol=1e-3)
    cb = C.to(torch.bfloat16).double()
    dd = ref.pairwise_sqdist(lo.x[:, :d].double(), cb, exact=True)
    top = dd.topk(2, largest=False).values
    scale = (lo.x[:, :d].double() ** 2).sum(1) + (cb * cb).sum(1).max()
    assert ((d2.double() - top[:, 1]).abs() <= 1e-5 * scale + 1e-3).all()
    assert (d2 >= d1).all()
    g = torch.Generator(device=gpu).manual_seed(3)
    idx = torch.randint(n, (n // 3,), generator=g, device=gpu, dtype=torch.int32)
    li = torch.empty(n // 3, dtype=torch.int32, device=gpu)
    e1 = torch.empty(n // 3, dtype=torch.float32, device=gpu)
    e2 = torch.empty(n // 3, dtype=torch.float32, device=gpu)
    ops.assign_bf16_top2(lo.x, idx, lo.cm2, lo.cnorm, li, e1, e2)
    assert torch.equal(li, lab[idx.long()]) and torch.equal(e2, d2[idx.long()])


@pytest.mark.parametrize("off", [0, 1])  # 1: unaligned views -> the scalar filter path
def test_bounds_filter_and_scatter(gpu, off):
    from tensorflow_distributed_clustering_amd import _native
    ops = _native.require()
    n, k = 100_003, 50
    g = torch.Generator(device=gpu).manual_seed(0)
    labels = torch.randint(k, (n + off,), generator=g, device=gpu, dtype=torch.int32)[off:]
    ub = torch.rand(n + off, generator=g, device=gpu)[off:]
    lb = ub + torch.rand(n, generator=g, device=gpu) * 0.5
    lb = torch.cat([lb[:off], lb])[off:] if off else lb
    drift = torch.rand(k, generator=g, device=gpu) * 0.1
    maxd = drift.max().reshape(1)
    ub2, lb2 = ub + drift[labels.long()], lb - maxd
    want = (~(ub2 * 1.001 < lb2)).nonzero().flatten()
    active = torch.empty(n, dtype=torch.int32, device=gpu)
    cnt = torch.zeros(2, dtype=torch.int32, device=gpu)
    ops.bounds_filter(labels, ub, lb, drift, maxd, 1e-3, active, cnt[0:1])
    m = int(cnt[0])
    assert m == want.numel() and torch.equal(active[:m].sort().values.long(), want)
    torch.testing.assert_close(ub, ub2)
    torch.testing.assert_close(lb, lb2)
    act = active[:m]
    blab = torch.where(act % 3 == 0, (labels[act.long()] + 1) % k, labels[act.long()])
    d1 = torch.rand(m, generator=g, device=gpu)
    d2 = d1 + 1
    moved = torch.empty(3, m, dtype=torch.int32, device=gpu)
    old = labels.clone()
    ops.bounds_scatter(act, cnt[0:1], blab, d1, d2, labels, ub, lb, moved[0], moved[1], moved[2],
                       cnt[1:2])
    mv = int(cnt[1])
    chg = act[(blab != old[act.long()])]
    assert mv == chg.numel()
    order = moved[0, :mv].sort()
    assert torch.equal(order.values, chg.sort().values)
    assert torch.equal(moved[1, :mv], old[moved[0, :mv].long()])
    assert torch.equal(moved[2, :mv], labels[moved[0, :mv].long()])
    assert torch.equal(labels[act.long()], blab)
    torch.testing.assert_close(ub[act.long()], d1.sqrt())


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
@pytest.mark.parametrize("n,d,k", [(5000, 96, 100), (4001, 128, 1000), (3000, 256, 130),
                                   (2000, 768, 257), (1500, 33, 65)])
def test_assign_exact_wide_d(gpu, dt, n, d, k):
    """Exact tiled assignment for wide D (replaces the library GEMM): difference-form
    distances, labels at the exact minimum, min distances to rounding."""
    from tensorflow_distributed_clustering_amd import _native
    ops = _native.require()
    x64, c64 = _bf16_case(n, d, k, "cpu", seed=n + d)
    x64, c64 = x64.double(), c64.double()
    x, c = x64.to(dt).to(gpu), c64.to(dt).to(gpu)
    labels = torch.full((n,), -1, dtype=torch.int32, device=gpu)
    mind = torch.zeros(n, dtype=dt, device=gpu)
    ops.assign_exact(x, c, labels, mind)
    rel = 1e-13 if dt == torch.float64 else 2e-6
    best = _check_labels(x.double().cpu(), c.double().cpu(), labels.cpu(), rel=rel)
    torch.testing.assert_close(mind.double().cpu(), best, rtol=1e-12 if dt == torch.float64 else 1e-5,
                               atol=1e-9)


@pytest.mark.parametrize("dtype,d,backend,exact", [("fp64", 48, "hip_x3_mfma", "auto"),
                                                   ("fp32", 96, "hip_x3_mfma", "auto"),
                                                   ("fp64", 48, "hip_exact_tiled", "simt"),
                                                   ("fp32", 96, "hip_exact_tiled", "simt"),
                                                   ("bf16", 768, "hip_bf16_wide", "auto"),
                                                   ("bf16", 900, "hip_bf16_wide", "auto"),
                                                   ("bf16", 1100, "hip_exact_tiled", "auto")])
def test_wide_d_lloyd_is_native(gpu, dtype, d, backend, exact):
    """fp64 D > 32 and fp32 D > 64 run native exact-argmin kernels (no library GEMM): the
    bf16x3 MFMA path with its exact re-check by default, the difference-form SIMT tiles
    with exact_assign='simt'; bf16 runs the wide MFMA kernel up to D=1024, above it the
    exact tiles."""
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
    x = gaussian_blobs(20000, d, 20, seed=3, dtype=torch.float64, device=gpu)
    r = tdc.KMeans(tdc.ClusterConfig(n_clusters=20, max_iter=3, dtype=dtype, seed=2,
                                     exact_assign=exact)).fit(x).result_
    assert r.backend == backend
    mfma = backend == "hip_bf16_wide"
    # the MFMA path keeps the shard in bf16: the oracle clusters the same rounded rows
    xo = x.bfloat16().double() if mfma else x
    o = tdc.KMeans(tdc.ClusterConfig(n_clusters=20, max_iter=3, dtype="fp64", seed=2,
                                     backend="torch"), device="cpu").fit(xo.cpu()).result_
    if mfma:  # bf16 centroid operands: boundary rows may flip, the clustering is the same
        agree = (r.labels.cpu() == torch.as_tensor(o.labels).cpu()).float().mean().item()
        assert agree > 0.99, agree
        torch.testing.assert_close(torch.as_tensor(r.centers), torch.as_tensor(o.centers),
                                   rtol=0, atol=0.15)
    else:
        torch.testing.assert_close(torch.as_tensor(r.centers), torch.as_tensor(o.centers),
                                   rtol=1e-4, atol=1e-4)
