"""CLI compatibility with `scripts/distribuitedClustering.py` (golden header/row format,
validators, exit codes, multi-process launch, centroids/labels CSV outputs)."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "scripts", "distribuitedClustering.py")
HEADER = "method_name,seed,num_GPUs,K,n_obs,n_dim,setup_time,initialization_time,computation_time,n_iter"


@pytest.fixture(scope="module")
def data(tmp_path_factory):
    from tensorflow_distributed_clustering_amd.data.synth import make_data
    p = tmp_path_factory.mktemp("d") / "class-data.npz"
    make_data(str(p), 3000, 5, 1826273)
    return str(p)


def run_cli(*args, env=None):
    e = dict(os.environ)
    e["CUDA_VISIBLE_DEVICES"] = ""
    e["HIP_VISIBLE_DEVICES"] = ""
    e.update(env or {})
    return subprocess.run([sys.executable, SCRIPT, *args], capture_output=True, text=True,
                          env=e, timeout=300)


def base_args(data, log, method="distributedKMeans", gpus=1, extra=()):
    return ["--n_obs", "3000", "--n_dim", "5", "--K", "3", "--n_GPUs", str(gpus),
            "--n_max_iters", "20", "--seed", "123128", "--log_file", log,
            "--method_name", method, "--data_file", data, *extra]


def test_header_and_row(data, tmp_path):
    log = str(tmp_path / "log.csv")
    r = run_cli(*base_args(data, log, extra=["--device", "cpu"]))
    assert r.returncode == 0, r.stderr
    lines = open(log).read().splitlines()
    assert lines[0] == HEADER
    f = lines[1].split(",")
    assert f[:6] == ["distributedKMeans", "123128", "1", "3", "3000", "5"]
    assert all(float(v) >= 0 for v in f[6:9]) and f[9] == "20"
    assert "log_file =" in r.stdout


def test_fcm_two_ranks_and_outputs(data, tmp_path):
    log = str(tmp_path / "log.csv")
    cen = str(tmp_path / "c.csv")
    lab = str(tmp_path / "l.csv")
    r = run_cli(*base_args(data, log, "distributedFuzzyCMeans", 2,
                           ["--device", "cpu", "--centroids_out", cen, "--labels_out", lab]))
    assert r.returncode == 0, r.stderr
    row = open(log).read().splitlines()[1].split(",")
    assert row[0] == "distributedFuzzyCMeans" and row[2] == "2"
    c = np.loadtxt(cen, delimiter=",")
    assert c.shape == (3, 5)
    l = np.loadtxt(lab, dtype=np.int64)
    assert l.shape == (3000,) and l.min() >= 0 and l.max() < 3


def test_errors_recorded_like_reference(data, tmp_path):
    log = str(tmp_path / "log.csv")
    # K larger than N -> ValueError in init -> class name in the time columns, exit 1
    args = base_args(data, log, extra=["--device", "cpu"])
    args[args.index("--K") + 1] = "5000"
    r = run_cli(*args)
    assert r.returncode == 1
    row = open(log).read().splitlines()[1].split(",")
    assert row[6:9] == ["ValueError"] * 3 and row[9] == "20"


def test_validators(data, tmp_path):
    log = str(tmp_path / "log.csv")
    r = run_cli(*base_args(data, log, method="distributedKMeansX", extra=["--device", "cpu"]))
    assert r.returncode == 2 and "Invalid Method Name" in r.stderr
    r = run_cli(*base_args(str(tmp_path / "missing.npz"), log, extra=["--device", "cpu"]))
    assert r.returncode == 2 and "Data File not Found" in r.stderr
    r = run_cli(*base_args(data, log, gpus=0, extra=["--device", "cpu"]))
    assert r.returncode == 2 and "Non Positive" in r.stderr
    args = base_args(data, log, extra=["--device", "cpu"])
    args[args.index("--K") + 1] = "three"
    r = run_cli(*args)
    assert r.returncode == 2 and "Invalid Integer" in r.stderr


def test_same_result_one_and_two_ranks(data, tmp_path):
    outs = []
    for g in (1, 2):
        cen = str(tmp_path / f"c{g}.csv")
        r = run_cli(*base_args(data, str(tmp_path / "log.csv"), gpus=g,
                               extra=["--device", "cpu", "--init", "random", "--dtype", "fp64",
                                      "--centroids_out", cen]))
        assert r.returncode == 0, r.stderr
        outs.append(np.loadtxt(cen, delimiter=","))
    np.testing.assert_allclose(outs[0], outs[1], rtol=1e-12)


def test_num_batches_averages_fits_from_shared_init(data, tmp_path):
    """--num_batches N: reference batch mode (`distribuitedClustering.py:296-318`): N
    array_split batches clustered independently from ONE shared initial center set (built
    once, `:325`), centers averaged, times summed; each batch checkpoints to its own file."""
    from tensorflow_distributed_clustering_amd import ClusterConfig, KMeans
    from tensorflow_distributed_clustering_amd.data.npz import open_npz_member
    from tensorflow_distributed_clustering_amd.utils import checkpoint as ck
    import torch
    log = str(tmp_path / "log.csv")
    cen = str(tmp_path / "c.csv")
    path = str(tmp_path / "run.npz")
    r = run_cli(*base_args(data, log, gpus=2, extra=["--device", "cpu", "--num_batches", "3",
                                                     "--dtype", "fp64", "--centroids_out", cen,
                                                     "--checkpoint", path]))
    assert r.returncode == 0, r.stderr
    row = open(log).read().splitlines()[1].split(",")
    assert row[2] == "2" and all(float(v) >= 0 for v in row[6:9])
    got = np.loadtxt(cen, delimiter=",")
    x = np.asarray(open_npz_member(data, "X"))
    parts = np.array_split(x, 3)
    cfg = ClusterConfig(n_clusters=3, max_iter=20, dtype="fp64", seed=123128, init="kmeans++")
    c0 = KMeans(cfg.replace(max_iter=0)).fit(torch.from_numpy(parts[0].copy())).result_.init_centers
    want = [KMeans(cfg).fit(torch.from_numpy(p.copy()), init_centers_=c0).result_.centers
            for p in parts]
    np.testing.assert_allclose(got, np.mean(want, axis=0), rtol=1e-9, atol=1e-9)
    # per-batch checkpoints + the averaged result under the base path
    for b in range(3):
        assert ck.load(str(tmp_path / f"run_b{b}.npz")).n_iter >= 1
    avg = ck.load(path)
    assert avg.method == "batched-average" and avg.meta["num_batches"] == 3
    np.testing.assert_allclose(avg.centers, got, rtol=1e-12)


def test_update_mode_flag_same_fit(data, tmp_path):
    """--update full / delta (the moved-rows update between fp64 totals) and --deterministic
    reach the same centroids through the CLI."""
    outs = []
    for extra in (["--update", "full"], ["--update", "delta"], ["--deterministic"]):
        cen = str(tmp_path / f"c{len(outs)}.csv")
        r = run_cli(*base_args(data, str(tmp_path / "log.csv"),
                               extra=["--device", "cpu", "--dtype", "fp64", "--init", "random",
                                      "--centroids_out", cen, *extra]))
        assert r.returncode == 0, r.stderr
        outs.append(np.loadtxt(cen, delimiter=","))
    np.testing.assert_allclose(outs[1], outs[0], rtol=1e-10, atol=1e-10)
    np.testing.assert_allclose(outs[2], outs[0], rtol=1e-10, atol=1e-10)


def test_resolve_dtype_auto_follows_the_measured_routing():
    """--dtype auto: K-Means fp64 up to D = 1024; FCM fp64 on the small fused kernel
    (D <= 16) and on the fp64 matrix-core path (K >= 64, where fp32 is promoted from D = 64),
    fp32 SIMT tower in between."""
    from tensorflow_distributed_clustering_amd.cli import resolve_dtype
    assert resolve_dtype("auto", 1024, 128) == "fp64"
    assert resolve_dtype("auto", 64, 2048) == "fp32"
    fcm = "distributedFuzzyCMeans"
    assert resolve_dtype("auto", 3, 5, fcm) == "fp64"
    assert resolve_dtype("auto", 1024, 128, fcm) == "fp64"
    assert resolve_dtype("auto", 128, 768, fcm) == "fp64"
    assert resolve_dtype("auto", 64, 128, fcm) == "fp64"
    assert resolve_dtype("auto", 32, 128, fcm) == "fp32"
    assert resolve_dtype("bf16", 64, 128, fcm) == "bf16"
