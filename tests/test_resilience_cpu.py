"""Checkpoint / resume, fault injection, OOM-adaptive retry, deterministic update
(the reference had only an OOM retry that clustered batches
independently, and no checkpointing at all)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import tensorflow_distributed_clustering_amd as tdc
from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
from tensorflow_distributed_clustering_amd.ops import fixed_point_scale
from tensorflow_distributed_clustering_amd.ops import reference as ref
from tensorflow_distributed_clustering_amd.utils import checkpoint as ck
from tensorflow_distributed_clustering_amd.utils import faults

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(autouse=True)
def _clean_faults(monkeypatch):
    monkeypatch.delenv("TDC_FAULT", raising=False)
    faults._FIRED.clear()
    yield
    faults._FIRED.clear()


def test_checkpoint_roundtrip_no_pickle(tmp_path):
    p = str(tmp_path / "c.npz")
    c = np.random.default_rng(0).normal(size=(7, 3))
    ck.save(p, ck.Checkpoint("distributedKMeans", 5, c, meta={"x": 1}, arrays={"counts": np.arange(7)}))
    got = ck.load(p)
    assert got.n_iter == 5 and got.method == "distributedKMeans" and got.meta["x"] == 1
    np.testing.assert_array_equal(got.centers, c)
    np.testing.assert_array_equal(got.arrays["counts"], np.arange(7))
    with np.load(p, allow_pickle=False) as z:  # loadable without pickle
        assert set(z.files) >= {"centers", "meta_json", "arr_counts"}


@pytest.mark.parametrize("model", ["kmeans", "fcm"])
def test_crash_then_resume_matches_uninterrupted(tmp_path, monkeypatch, model):
    x = gaussian_blobs(4000, 3, 5, seed=3, dtype=torch.float64)
    cls = tdc.KMeans if model == "kmeans" else tdc.FuzzyCMeans
    base = tdc.ClusterConfig(n_clusters=5, max_iter=8, dtype="fp64", seed=2, fuzzifier=2.0)
    full = cls(base).fit(x).result_
    path = str(tmp_path / "run.npz")
    cfg = base.replace(checkpoint_path=path, checkpoint_every=1)
    monkeypatch.setenv("TDC_FAULT", "crash@3")
    with pytest.raises(faults.InjectedFault):
        cls(cfg).fit(x)
    assert ck.load(path).n_iter == 3
    monkeypatch.delenv("TDC_FAULT")
    res = cls(cfg.replace(resume=True)).fit(x).result_
    assert res.n_iter == 8
    np.testing.assert_allclose(res.centers, full.centers, rtol=1e-12, atol=1e-12)
    assert ck.load(path).n_iter == 8  # final checkpoint


def test_resume_rejects_mismatched_checkpoint(tmp_path):
    path = str(tmp_path / "run.npz")
    ck.save(path, ck.Checkpoint("distributedKMeans", 2, np.zeros((4, 3))))
    x = gaussian_blobs(500, 3, 5, seed=1, dtype=torch.float64)
    with pytest.raises(ValueError):
        tdc.KMeans(tdc.ClusterConfig(n_clusters=5, dtype="fp64", checkpoint_path=path,
                                     resume=True)).fit(x)


def test_minibatch_checkpoint_restores_counts(tmp_path, monkeypatch):
    x = gaussian_blobs(20000, 2, 4, seed=5, dtype=torch.float64)
    path = str(tmp_path / "mb.npz")
    cfg = tdc.ClusterConfig(n_clusters=4, max_iter=20, dtype="fp64", batch_size=500, seed=1,
                            checkpoint_path=path, checkpoint_every=5)
    monkeypatch.setenv("TDC_FAULT", "crash@10")
    with pytest.raises(faults.InjectedFault):
        tdc.MiniBatchKMeans(cfg).fit(x)
    saved = ck.load(path)
    assert saved.n_iter == 10 and saved.arrays["counts"].sum() == 10 * 500
    monkeypatch.delenv("TDC_FAULT")
    mb = tdc.MiniBatchKMeans(cfg.replace(resume=True)).fit(x)
    assert mb.result_.n_iter == 20
    assert mb.result_.counts.sum() == 20 * 500


def test_setup_oom_retries_streamed(monkeypatch, capsys):
    x = gaussian_blobs(5000, 4, 6, seed=7, dtype=torch.float64)
    cfg = tdc.ClusterConfig(n_clusters=6, max_iter=6, dtype="fp64", seed=4)
    ref_run = tdc.KMeans(cfg).fit(x).result_
    monkeypatch.setenv("TDC_FAULT", "oom@setup")
    res = tdc.KMeans(cfg).fit(x).result_
    assert res.streamed  # the retry streams the shard in halved chunks
    assert "retrying streamed with chunk_rows=1250" in capsys.readouterr().out
    np.testing.assert_allclose(res.centers, ref_run.centers, rtol=1e-12, atol=1e-12)


def test_setup_oom_gives_up_after_retries(monkeypatch):
    x = gaussian_blobs(500, 2, 3, seed=7, dtype=torch.float64)
    monkeypatch.setenv("TDC_FAULT", "oom@setup")
    # zero retries allowed -> the injected OOM surfaces
    with pytest.raises(Exception) as ei:
        tdc.KMeans(tdc.ClusterConfig(n_clusters=3, dtype="fp64", max_oom_retries=0)).fit(x)
    assert faults.is_oom(ei.value)


def test_fixed_point_scale_bounds_the_sums():
    """The deterministic update's int64 fixed point: 2^S with max|x| * N * 2^S < 2^61 (no
    per-cluster sum can overflow int64) and max|x| * 2^S <= 2^30 (every element's fixed
    point fits an int32), the largest such power of two (clamped)."""
    import math
    for m, n in [(15.0, 10_000_000), (1e-3, 100), (1e6, 10 ** 9), (0.0, 5), (7.5, 1),
                 (2.0, 2 ** 40)]:
        s = fixed_point_scale(m, n)
        mm = max(m, 1e-30)
        assert s == 2.0 ** round(math.log2(s))
        assert mm * n * s < 2.0 ** 61 and mm * s <= 2.0 ** 30
        if 2.0 ** -60 < s < 2.0 ** 60:  # not needlessly coarse: one of the bounds is tight
            assert mm * n * s * 4 >= 2.0 ** 61 or mm * s * 2 > 2.0 ** 30
    assert fixed_point_scale(15.0, 10_000_000) == 2.0 ** 26
    assert fixed_point_scale(2.0, 2 ** 40) == 2.0 ** 19  # the sum bound binds
    # fp64 rows: only the sum bound (int64 conversion), a much finer step
    assert fixed_point_scale(15.0, 10_000_000, elem32=False) == 2.0 ** 32
    for m, n in [(15.0, 10_000_000), (1e6, 10 ** 9)]:
        s = fixed_point_scale(m, n, elem32=False)
        assert m * n * s < 2.0 ** 61 and m * n * s * 4 >= 2.0 ** 61


def test_deterministic_cpu_fit_reproducible():
    x = gaussian_blobs(20000, 5, 6, seed=4, dtype=torch.float64)
    cfg = tdc.ClusterConfig(n_clusters=6, max_iter=6, dtype="fp64", deterministic=True)
    a = tdc.KMeans(cfg).fit(x).result_
    b = tdc.KMeans(cfg).fit(x).result_
    assert np.array_equal(a.centers, b.centers) and torch.equal(a.labels, b.labels)


def test_cli_checkpoint_resume(tmp_path):
    data = tmp_path / "d.npz"
    X = gaussian_blobs(3000, 3, 4, seed=9, dtype=torch.float64).numpy()
    np.savez(data, X=X, Y=np.zeros(3000))
    log = tmp_path / "log.csv"
    ckp = tmp_path / "c.npz"
    cen = tmp_path / "cent.csv"
    cmd = [sys.executable, os.path.join(ROOT, "scripts", "distribuitedClustering.py"),
           "--n_obs=3000", "--n_dim=3", "--K=4", "--n_GPUs=1", "--n_max_iters=6", "--seed=3",
           f"--log_file={log}", "--method_name=distributedKMeans", f"--data_file={data}",
           "--device=cpu", f"--checkpoint={ckp}", "--checkpoint_every=2", f"--centroids_out={cen}"]
    env = dict(os.environ, TDC_FAULT="crash@4")
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=300)
    assert "InjectedFault" in (r.stdout + r.stderr)
    assert ck.load(str(ckp)).n_iter == 4
    env.pop("TDC_FAULT")
    r = subprocess.run(cmd + ["--resume"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "resuming from" in r.stdout
    rows = open(log).read().strip().splitlines()
    assert rows[1].split(",")[6] == "InjectedFault" and rows[2].split(",")[-1] == "6"


def _oom_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank), TDC_FAULT="oom@setup:1")
    torch.set_num_threads(1)
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.parallel import dist as D
    D._COMM = None
    comm = D.init_comm("cpu")
    s, e = comm.shard(4001)
    x = gaussian_blobs(e - s, 3, 5, seed=2, row_offset=s, dtype=torch.float64)
    cfg = tdc.ClusterConfig(n_clusters=5, max_iter=5, dtype="fp64", seed=1)
    r = tdc.KMeans(cfg, comm).fit(x, n_global=4001, row_offset=s).result_
    if rank == 0:
        q.put((r.centers, r.streamed))
    D.destroy_comm()


def test_oom_on_one_rank_retries_on_all_ranks():
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_oom_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    centers, streamed = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert streamed  # rank 0 did not OOM itself but followed the collective retry
    x = gaussian_blobs(4001, 3, 5, seed=2, dtype=torch.float64)
    single = tdc.KMeans(tdc.ClusterConfig(n_clusters=5, max_iter=5, dtype="fp64", seed=1)).fit(x)
    np.testing.assert_allclose(centers, single.result_.centers, rtol=1e-10, atol=1e-10)


def _midrun_worker(rank, world, port, method, fault, q):
    env = dict(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
               RANK=str(rank), LOCAL_RANK=str(rank))
    if fault:
        env["TDC_FAULT"] = fault
    os.environ.update(env)
    torch.set_num_threads(1)
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.parallel import dist as D
    D._COMM = None
    comm = D.init_comm("cpu")
    s, e = comm.shard(4001)
    x = gaussian_blobs(e - s, 3, 5, seed=2, row_offset=s, dtype=torch.float64)
    cfg = tdc.ClusterConfig(n_clusters=5, max_iter=6, dtype="fp64", seed=1, init="first_k",
                            fuzzifier=2.0)
    model = (tdc.KMeans if method == "kmeans" else tdc.FuzzyCMeans)(cfg, comm)
    r = model.fit(x, n_global=4001, row_offset=s).result_
    if rank == 0:
        q.put((r.centers, r.streamed, r.n_iter))
    D.destroy_comm()


def _run_midrun(method, fault):
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_midrun_worker, args=(r, 2, port, method, fault, q))
             for r in range(2)]
    for p in procs:
        p.start()
    out = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return out


_MIDRUN_REF = {}


@pytest.mark.parametrize("method", ["kmeans", "fcm"])
@pytest.mark.parametrize("fault", ["oom@3:1", "oom@5:1"])
def test_mid_run_oom_on_one_rank_continues_streamed(method, fault):
    """TDC_FAULT=oom@3:1: rank 1 runs out of memory inside iteration 3.  The flag rides in
    the packed all-reduce, both ranks roll back to the centroids before iteration 3 and
    finish on a streamed engine with the same result as an undisturbed run (the reference
    restarted the whole run with doubled batches, scripts/distribuitedClustering.py:357-360).
    oom@5 of 6: a step within the flag lag of the end, caught by the final check."""
    if method not in _MIDRUN_REF:
        _MIDRUN_REF[method] = _run_midrun(method, "")
    c_ref, streamed_ref, it_ref = _MIDRUN_REF[method]
    c, streamed, it = _run_midrun(method, fault)
    assert not streamed_ref and streamed and it == it_ref == 6
    np.testing.assert_allclose(c, c_ref, rtol=1e-10, atol=1e-10)


def test_fcm_setup_oom_retries_streamed(monkeypatch, capsys):
    monkeypatch.setenv("TDC_FAULT", "oom@setup")
    from tensorflow_distributed_clustering_amd.utils import faults
    faults._FIRED.clear()
    x = gaussian_blobs(3000, 3, 4, seed=5, dtype=torch.float64)
    cfg = tdc.ClusterConfig(n_clusters=4, max_iter=5, dtype="fp64", init="first_k", fuzzifier=2.0)
    r = tdc.FuzzyCMeans(cfg).fit(x.numpy()).result_
    assert r.streamed and "retrying streamed" in capsys.readouterr().out
    monkeypatch.delenv("TDC_FAULT")
    ref = tdc.FuzzyCMeans(cfg).fit(x.numpy()).result_
    np.testing.assert_allclose(r.centers, ref.centers, rtol=1e-10, atol=1e-10)


def test_cli_log_every_profile_and_timeout_flags(tmp_path):
    data = tmp_path / "d.npz"
    X = gaussian_blobs(3000, 3, 4, seed=9, dtype=torch.float64).numpy()
    np.savez(data, X=X, Y=np.zeros(3000))
    ext, prof = tmp_path / "e.jsonl", tmp_path / "prof"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "distribuitedClustering.py"),
                        "--n_obs=3000", "--n_dim=3", "--K=4", "--n_GPUs=1", "--n_max_iters=6",
                        "--seed=3", f"--log_file={tmp_path / 'l.csv'}",
                        "--method_name=distributedKMeans", f"--data_file={data}", "--device=cpu",
                        "--log_every=3", f"--extended_log={ext}", f"--torch_profile={prof}",
                        "--collective_timeout=120"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "[kmeans] iter 3 max centroid shift^2" in r.stdout and "inertia" in r.stdout
    import json
    hist = json.loads(ext.read_text().strip())["history"]
    assert [h["iter"] for h in hist] == [3, 6] and all(h["inertia"] > 0 for h in hist)
    assert (prof / "trace_rank0.json").exists() and (prof / "kernels_rank0.txt").exists()


def _resume_worker(rank, world, port, path, crash, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    if crash:
        os.environ["TDC_FAULT"] = "crash@3"
    else:
        os.environ.pop("TDC_FAULT", None)
    torch.set_num_threads(1)
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.parallel import dist as D
    from tensorflow_distributed_clustering_amd.utils import faults as F
    D._COMM = None
    comm = D.init_comm("cpu")
    s, e = comm.shard(6001)
    x = gaussian_blobs(e - s, 3, 5, seed=4, row_offset=s, dtype=torch.float64)
    cfg = tdc.ClusterConfig(n_clusters=5, max_iter=8, dtype="fp64", seed=2,
                            checkpoint_path=path, checkpoint_every=1, resume=not crash)
    try:
        r = tdc.KMeans(cfg, comm).fit(x, n_global=6001, row_offset=s).result_
        if rank == 0:
            q.put(("ok", r.centers))
    except F.InjectedFault:
        if rank == 0:
            q.put(("crashed", None))
    D.destroy_comm()


def _world2(path, crash):
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_resume_worker, args=(r, 2, port, path, crash, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
    return out


def test_distributed_crash_and_resume(tmp_path):
    path = str(tmp_path / "dist.npz")
    status, _ = _world2(path, crash=True)
    assert status == "crashed" and ck.load(path).n_iter == 3
    status, centers = _world2(path, crash=False)
    assert status == "ok"
    x = gaussian_blobs(6001, 3, 5, seed=4, dtype=torch.float64)
    full = tdc.KMeans(tdc.ClusterConfig(n_clusters=5, max_iter=8, dtype="fp64", seed=2)).fit(x)
    np.testing.assert_allclose(centers, full.result_.centers, rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("model", ["kmeans", "fcm"])
def test_mid_run_oom_releases_the_old_engine(monkeypatch, capsys, model):
    """After a mid-run OOM the engine that failed (its device shard, operand tables, graph
    pool) is garbage before the streamed engine is built: fit keeps only weak references
    to it, and those are dead once the fit returns."""
    x = gaussian_blobs(3000, 3, 4, seed=5, dtype=torch.float64)
    cfg = tdc.ClusterConfig(n_clusters=4, max_iter=6, dtype="fp64", init="first_k",
                            fuzzifier=2.0)
    cls = tdc.KMeans if model == "kmeans" else tdc.FuzzyCMeans
    ref_run = cls(cfg).fit(x.numpy()).result_
    monkeypatch.setenv("TDC_FAULT", "oom@3")
    m = cls(cfg)
    r = m.fit(x.numpy()).result_
    assert r.streamed and "continuing streamed" in capsys.readouterr().out
    assert len(m._retired) == 1 and all(w() is None for w in m._retired)
    np.testing.assert_allclose(r.centers, ref_run.centers, rtol=1e-10, atol=1e-10)
