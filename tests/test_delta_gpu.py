"""Delta centroid update of plain Lloyd (ClusterConfig.update='delta', csrc/update_sorted.hip
delta_* + centroids.hip finalize_delta) against a plain-PyTorch fp64 reference of the same
op, and whole fits against the full re-summing update (reference per-iteration update:
scripts/distribuitedClustering.py:237-263)."""
import numpy as np
import pytest
import torch

import tensorflow_distributed_clustering_amd as tdc
from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
from tensorflow_distributed_clustering_amd.ops import (DC_EVENTS, DC_ITER, DC_MODE, DC_NEXT,
                                                        DC_PREVOK, DC_WORDS)

pytestmark = pytest.mark.gpu


def _ops():
    from tensorflow_distributed_clustering_amd import _native
    return _native.require()


@pytest.mark.parametrize("xdt,acc,split", [(torch.bfloat16, torch.float32, True),
                                           (torch.float32, torch.float64, False),
                                           (torch.float64, torch.float64, False)])
@pytest.mark.parametrize("n,d,k,off", [(50_003, 128, 1024, 0), (9000, 37, 100, 0),
                                       (70_000, 64, 8192, 0), (30_001, 128, 512, 1),
                                       (90_000, 48, 20_000, 0), (40_000, 32, 65_536, 1)])
def test_delta_update_op_vs_torch(gpu, xdt, acc, split, n, d, k, off):
    """off = 1: labels / prev are views one element into their buffers (not 16-B aligned:
    the diff kernel's scalar-load form)."""
    ops = _ops()
    g = torch.Generator().manual_seed(n + k)
    x = torch.randn(n, d, generator=g, dtype=torch.float64).to(xdt).to(gpu)
    prev = torch.randint(0, k, (n + off,), generator=g, dtype=torch.int32)
    labels = prev.clone()
    mv = torch.rand(n + off, generator=g) < 0.07
    labels[mv] = torch.randint(0, k, (int(mv.sum()),), generator=g, dtype=torch.int32)
    prev, labels = prev.to(gpu)[off:], labels.to(gpu)[off:]
    work = torch.zeros(int(ops.delta_workspace(n, k)), dtype=torch.int32, device=gpu)
    ctrl = torch.zeros(DC_WORDS, dtype=torch.int32, device=gpu)
    buf = torch.full((k * d + 3 * k + 1,), 7.0, dtype=acc, device=gpu)  # garbage: zeroed first
    sums, counts = buf[: k * d].view(k, d), buf[k * d: k * d + k]
    hi = buf[k * d + k: k * d + 2 * k] if split else None
    lo = buf[k * d + 2 * k: k * d + 3 * k] if split else None
    moved = buf[-1:]
    x64 = x.double()
    for full in (0, 1):
        ctrl[DC_NEXT] = full
        p0 = prev.clone()
        ops.delta_update(x, labels, prev, sums, counts, work, ctrl, hi, lo, moved, buf)
        torch.cuda.synchronize()
        new, old = labels.long(), p0.long()
        chg = new != old
        if full:
            rs = torch.zeros(k, d, dtype=torch.float64, device=gpu).index_add_(0, new, x64)
            rc = torch.bincount(new, minlength=k).double()
        else:
            i = torch.nonzero(chg).flatten()
            rs = torch.zeros(k, d, dtype=torch.float64, device=gpu)
            rs.index_add_(0, new[i], x64[i]).index_add_(0, old[i], -x64[i])
            rc = (torch.bincount(new[i], minlength=k) - torch.bincount(old[i], minlength=k)).double()
        tol = 1e-9 if xdt == torch.float64 else 1e-3  # fp32 partial registers otherwise
        torch.testing.assert_close(sums.double(), rs, rtol=tol, atol=tol)
        torch.testing.assert_close(counts.double(), rc)
        if split:
            torch.testing.assert_close(hi.double() * 4096 + lo.double(), rc)
        assert float(moved) == float(chg.sum())
        assert torch.equal(prev, labels)  # prev = labels on return
        assert int(ctrl[DC_MODE]) == full
        assert int(ctrl[DC_EVENTS]) == (n if full else 2 * int(chg.sum()))
        # second call: no row changed any more -> an all-zero delta
        if not full:
            ctrl[DC_NEXT] = 0
            ops.delta_update(x, labels, prev, sums, counts, work, ctrl, hi, lo, moved, buf)
            torch.cuda.synchronize()
            assert float(sums.abs().max()) == 0.0 and float(counts.abs().max()) == 0.0
            assert float(moved) == 0.0
            prev.copy_(p0)  # restore the moved rows for the full pass


def test_delta_finalize_op(gpu):
    """G += deltas (delta mode) / G = partials (full mode), C = G means with bf16 operand
    prep, and the device-side choice of the next step's mode."""
    ops = _ops()
    k, d, kp = 70, 96, 128
    g = torch.Generator().manual_seed(3)
    G0 = torch.rand(k * d + k, generator=g, dtype=torch.float64) * 10
    G0[k * d:] = torch.randint(0, 50, (k,), generator=g).double()
    G0[k * d + 5] = 0.0  # empty cluster: keep policy
    dsum = torch.randn(k * d, generator=g, dtype=torch.float64).float()
    dcnt = torch.randint(-3, 4, (k,), generator=g).float()
    dcnt[5] = 0.0
    C = torch.randn(k, d, generator=g).float()
    G = G0.clone().to(gpu)
    Cg = C.clone().to(gpu)
    cm2 = torch.zeros(kp, 128, dtype=torch.bfloat16, device=gpu)
    cnorm = torch.zeros(kp, dtype=torch.float32, device=gpu)
    ctrl = torch.zeros(DC_WORDS, dtype=torch.int32, device=gpu)
    stats = torch.zeros(4, dtype=torch.float64, device=gpu)
    moved = torch.tensor([123.0], device=gpu)
    ctrl[DC_MODE], ctrl[DC_PREVOK], ctrl[DC_ITER] = 0, 1, 4
    ops.delta_finalize(dsum.to(gpu), dcnt.to(gpu), None, None, moved, G, Cg, 0, None, cm2, cnorm,
                       ctrl, stats, 5, 100.0)
    torch.cuda.synchronize()
    Gr = G0.clone()
    Gr[: k * d] += dsum.double()
    Gr[k * d:] += dcnt.double()
    torch.testing.assert_close(G.cpu(), Gr)
    cnt = Gr[k * d:]
    want = torch.where(cnt[:, None] > 0, Gr[: k * d].view(k, d) / cnt[:, None], C.double()).float()
    torch.testing.assert_close(Cg.cpu(), want)
    cb = want.to(torch.bfloat16)
    assert torch.equal(cm2[:k, :d].cpu(), (-2 * cb.float()).to(torch.bfloat16))
    assert float(cnorm[k]) > 1e37  # padding rows never win
    # ITER 4 -> 5: refresh every 5 steps -> the next step is full
    assert int(ctrl[DC_ITER]) == 5 and int(ctrl[DC_NEXT]) == 1
    assert stats.tolist() == [123.0, 1.0, 0.0, 1.0]
    # full mode replaces G; moved above theta_n also asks for a full step
    ctrl[DC_MODE] = 1
    ops.delta_finalize(dsum.to(gpu), dcnt.abs().to(gpu), None, None, moved, G, Cg, 0, None, cm2,
                       cnorm, ctrl, stats, 0, 100.0)
    torch.cuda.synchronize()
    torch.testing.assert_close(G[: k * d].cpu(), dsum.double())
    assert int(ctrl[DC_NEXT]) == 1  # 123 moved > theta_n = 100
    ops.delta_finalize(dsum.to(gpu), dcnt.abs().to(gpu), None, None, moved, G, Cg, 0, None, cm2,
                       cnorm, ctrl, stats, 0, 1000.0)
    torch.cuda.synchronize()
    assert int(ctrl[DC_NEXT]) == 0
    assert stats.tolist()[2:] == [2.0, 3.0]


def _fit(x, k, iters, dtype="bf16", **kw):
    cfg = tdc.ClusterConfig(n_clusters=k, max_iter=iters, dtype=dtype, init="random", seed=3,
                            **kw)
    km = tdc.KMeans(cfg).fit(x)
    return km.result_, km.engine_


def test_delta_matches_full_50_iterations(gpu):
    """Headline-like shape, 50 iterations (with a refresh at 32): the delta update reaches
    the full update's centroids (1e-5) and labels (>= 0.999)."""
    n, d, k = 400_000, 128, 1024
    x = gaussian_blobs(n, d, k, seed=4, dtype=torch.bfloat16, device=gpu)
    rf, ef = _fit(x, k, 50, update="full")
    rd, ed = _fit(x, k, 50, update="delta")
    assert ef.update_mode == "full" and ed.update_mode == "delta"
    st = ed.update_stats()
    # warm-up step + 50: the warm-up is full, the delta state is reset after it (timed
    # iteration 1 re-sums every row, as the reference's first iteration), then every 32 steps
    assert st["steps"] == 51 and st["full_steps"] == 3, st
    assert st["moved_rows"] / max(1.0, st["moved_steps"]) < 0.05 * n
    np.testing.assert_allclose(rd.centers, rf.centers, rtol=1e-5, atol=1e-5)
    assert (rd.labels == rf.labels).float().mean().item() >= 0.999
    assert rd.counts.sum() == rf.counts.sum() == n
    assert np.abs(rd.counts - rf.counts).max() <= 1e-3 * n
    assert rd.inertia == pytest.approx(rf.inertia, rel=1e-5)


@pytest.mark.parametrize("dtype,n,d,k", [
    ("bf16", 100_000, 64, 16),      # LDS-privatised full update
    ("bf16", 60_000, 384, 256),     # wide-D MFMA assign
    ("fp8", 40_000, 256, 300),      # fp8 assign, update from the bf16 shard, re-quantise
    ("fp32", 50_000, 100, 128),     # exact tiled assign
    ("fp64", 50_000, 20, 50),       # SIMT assign, fp64 rows
    ("fp8", 150_000, 256, 12_000),  # K > 8192: global histograms / cursors
])
def test_delta_matches_full_other_paths(gpu, dtype, n, d, k):
    tdt = {"bf16": torch.bfloat16, "fp8": torch.bfloat16, "fp32": torch.float32,
           "fp64": torch.float64}[dtype]
    x = gaussian_blobs(n, d, k, seed=6, dtype=tdt, device=gpu)
    rf, _ = _fit(x, k, 12, dtype=dtype, update="full")
    rd, ed = _fit(x, k, 12, dtype=dtype, update="delta", delta_refresh=5)
    assert ed.update_mode == "delta"
    tol = 1e-9 if dtype == "fp64" else 2e-5
    np.testing.assert_allclose(rd.centers, rf.centers, rtol=tol, atol=tol)
    assert (rd.labels == rf.labels).float().mean().item() >= 0.999


def test_delta_theta_fallback_and_nan_policy(gpu):
    """theta = 0: every step after one that moved a row is a full step (the device-side
    fallback), with the same result; the 'nan' policy on a globally empty cluster."""
    n, d, k = 80_000, 128, 200
    x = gaussian_blobs(n, d, 150, seed=8, dtype=torch.bfloat16, device=gpu)
    rf, _ = _fit(x, k, 10, update="full", empty_cluster="nan")
    rd, ed = _fit(x, k, 10, update="delta", delta_theta=0.0, delta_refresh=0,
                  empty_cluster="nan")
    st = ed.update_stats()
    assert st["full_steps"] >= 2
    assert np.array_equal(np.isnan(rd.centers), np.isnan(rf.centers))
    ok = ~np.isnan(rf.centers)
    np.testing.assert_allclose(rd.centers[ok], rf.centers[ok], rtol=1e-5, atol=1e-5)


def test_delta_graph_replay_equals_eager(gpu):
    """The whole delta step (mode decided on the device) replays from a hipGraph."""
    from tensorflow_distributed_clustering_amd.models.kmeans import LloydEngine
    from tensorflow_distributed_clustering_amd.parallel.dist import local_comm
    n, d, k = 150_000, 128, 512
    x = gaussian_blobs(n, d, k, seed=9, dtype=torch.bfloat16, device=gpu)
    cfg = tdc.ClusterConfig(n_clusters=k, max_iter=10, dtype="bf16", seed=9, delta_refresh=4)
    out = []
    for graph in (False, True):
        eng = LloydEngine(x, cfg, local_comm(gpu), n, 0)
        if graph:
            eng.capture()
        for _ in range(10):
            eng.step()
        torch.cuda.synchronize()
        out.append((eng.C.cpu().numpy(), eng.update_stats()))
    np.testing.assert_allclose(out[1][0], out[0][0], rtol=1e-5, atol=1e-5)
    # capture() runs one eager warm-up step first: one step more on the graph engine
    assert out[1][1]["steps"] == out[0][1]["steps"] + 1
