"""bench.py contract (driver-facing): one JSON line from rank 0, whole-job value, torchrun
launch with one rank per device (gloo ranks on CPU here)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config"}


def _run(args, timeout=600):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                       capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("gpus", [1, 2])
@pytest.mark.parametrize("scaling", ["strong", "weak"])
def test_bench_json_contract(gpus, scaling):
    d = _run(["--gpus", str(gpus), "--steps", "3", "--warmup", "1", "--n-per-gpu", "20000",
              "--k", "16", "--dim", "8", "--dtype", "fp32", "--scaling", scaling])
    assert KEYS <= set(d)
    n = 20000 * gpus if scaling == "weak" else 20000
    assert d["n_gpus"] == gpus and d["steps"] == 3 and d["warmup"] == 1
    assert d["config"]["global_batch"] == n and d["config"]["parallelism"] == f"dp{gpus}"
    assert d["scaling"] == scaling and d["higher_is_better"] is True
    # whole-job value = global points per step / step time
    assert d["value"] == pytest.approx(n / (d["ms_per_step"] / 1e3), rel=1e-6)
    if gpus > 1:  # per-phase times (max over ranks) ride along at world > 1
        assert set(d["phase_ms"]) == {"zero", "assign", "update", "allreduce", "finalize"}
    # the update mode of the timed steps and the correctness witness (after the timing)
    assert d["update"]["mode"] == "delta" and 0.0 <= d["update"]["moved_frac_mean"] <= 1.0
    # the timed steps are iterations 1..K from the init (the reference's computation_time):
    # the delta update's first full step is inside the window; the steady state rides along
    assert d["timed_from"] == "init" and d["update"]["full_steps_timed"] >= 1
    assert d["ms_per_step_steady"] > 0 and "moved_frac_mean" in d["update"]["steady"]
    assert d["check"]["sample_rows"] == 20000 if n == 20000 else d["check"]["sample_rows"] > 0
    assert d["check"]["agree_fp64_sample"] >= 0.99 and d["check"]["inertia"] > 0


def test_bench_update_full_and_witness():
    """--update full times the re-summing update; both modes report the witness, and the
    fits agree."""
    args = ["--steps", "4", "--warmup", "1", "--n-per-gpu", "40000", "--k", "12", "--dim", "6",
            "--dtype", "fp32"]
    dd = _run(args)
    df = _run(args + ["--update", "full"])
    assert dd["update"]["mode"] == "delta" and df["update"]["mode"] == "full"
    assert df["check"]["agree_fp64_sample"] >= 0.99
    assert dd["check"]["inertia"] == pytest.approx(df["check"]["inertia"], rel=1e-9)
    # an opt-in variant is named in the config (--fp8-recheck: the fp8 kernels only)
    dr = _run(args + ["--fp8-recheck", "0.05"])
    assert dr["config"]["fp8_recheck"] == 0.05 and "fp8_recheck" not in dd["config"]


def test_bench_settle_warmup_same_steps_on_every_rank():
    """--settle-ms: the warm-up keeps stepping until it has run that long, every rank the
    same number of steps (a mismatch would hang the collectives), and the timed steps still
    start from the init (the same fit as with exactly W warm-up steps)."""
    args = ["--gpus", "2", "--steps", "3", "--warmup", "2", "--n-per-gpu", "40000", "--k", "12",
            "--dim", "6", "--dtype", "fp32", "--scaling", "weak"]
    d0 = _run(args)
    d1 = _run(args + ["--settle-ms", "300"])
    assert d0["warmup_steps_run"] == 2 and d1["warmup"] == 2
    assert d1["warmup_steps_run"] > 2 and d1["warmup_ms"] >= 300
    assert d1["timed_from"] == "init"
    assert d1["check"]["inertia"] == pytest.approx(d0["check"]["inertia"], rel=1e-9)


def test_bench_headline_is_strong_scaling_at_10m(tmp_path):
    """The default preset measures BASELINE.json's metric: N = 10M points in TOTAL, split
    over the ranks (strong scaling), so --gpus 1/2/4 time the same problem and reach the
    same centroids (gloo ranks on CPU; D and K reduced so the CPU fp32 path is quick)."""
    cs = {}
    for g in (1, 2, 4):
        out = tmp_path / f"c{g}.npy"
        d = _run(["--gpus", str(g), "--steps", "2", "--warmup", "1", "--k", "16", "--dim", "8",
                  "--dtype", "fp32", "--centers-out", str(out)], timeout=900)
        assert d["scaling"] == "strong" and d["preset"] == "headline"
        assert d["config"]["N"] == 10_000_000 and d["config"]["global_batch"] == 10_000_000
        assert d["config"]["points_per_gpu"] == 10_000_000 // g
        cs[g] = np.load(out)
    for g in (2, 4):
        np.testing.assert_allclose(cs[g], cs[1], rtol=1e-4, atol=1e-4)


def test_bench_fcm_and_minibatch_presets():
    d = _run(["--preset", "ref25m_fcm", "--n-per-gpu", "30000", "--steps", "2", "--warmup", "1"])
    assert d["config"]["model"] == "fuzzy-cmeans" and d["dtype"] == "fp64"
    # FCM witness: one step of the engine's tower vs the fp64 oracle on the sample rows
    assert d["check"]["fcm_centroid_rel_err"] < 1e-9 and d["check"]["fcm_weight_sum_rel_err"] < 1e-9
    assert d["check"]["sample_rows"] == 30000 and "fp64" in d["precision"]
    # ... also from the init centroids (random rows: the exact oracle's zero distances)
    ini = d["check"]["at_init"]
    assert ini["fcm_centroid_rel_err"] < 1e-9 and ini["fcm_weight_sum_rel_err"] < 1e-9
    assert ini["ws_spread"] > 0 and d["check"]["final_ws_spread"] >= 0
    d = _run(["--preset", "minibatch1b", "--n-per-gpu", "50000", "--k", "32", "--batch-size", "4096",
              "--steps", "2", "--warmup", "1", "--dtype", "fp32"])
    assert d["config"]["model"] == "kmeans-minibatch" and d["config"]["global_batch"] == 4096


def test_bench_host_source():
    """--source host: the shard lives in host memory and goes through HostSource (streamed
    Lloyd with chunk_rows, and mini-batch chunks); the JSON says so and carries the
    stream geometry (on a GPU box it also reports the achieved H2D GB/s)."""
    d = _run(["--n-per-gpu", "30000", "--k", "16", "--dim", "8", "--dtype", "fp32", "--steps", "2",
              "--warmup", "1", "--source", "host"])
    assert "HOST memory" in d["data"] and d["source"]["rows"] == 30000
    assert d["config"]["model"] == "kmeans-lloyd" and d["source"]["chunk_rows"] > 0
    d = _run(["--preset", "minibatch1b", "--n-per-gpu", "30000", "--k", "16", "--batch-size", "4096",
              "--steps", "3", "--warmup", "1", "--dtype", "fp32", "--source", "host"])
    assert d["config"]["model"] == "kmeans-minibatch" and d["source"]["chunk_rows"] == 4096


def test_bench_from_init_equals_fit():
    """Rewinding to the init after the warm-up: the centroids after K timed steps equal a
    fit of K iterations from the same init (warm-up count does not matter)."""
    import tempfile
    outs = []
    with tempfile.TemporaryDirectory() as td:
        for w in (0, 3):
            out = os.path.join(td, f"c{w}.npy")
            d = _run(["--steps", "4", "--warmup", str(w), "--n-per-gpu", "30000", "--k", "12",
                      "--dim", "6", "--dtype", "fp32", "--no-steady", "--centers-out", out])
            assert d["timed_from"] == "init" and d["ms_per_step_steady"] is None
            outs.append(np.load(out))
    np.testing.assert_allclose(outs[0], outs[1], rtol=1e-12, atol=1e-12)


def test_fcm10m_preset_keeps_structure():
    """The fcm10m preset's data (blobs at cluster_std 0.25) keeps cluster structure under
    m = 2 FCM at D = 128, K = 1024: the final-state witness is informative
    (final_ws_spread > 0.1, per-cluster weight sums differ) instead of the collapsed,
    trivially exact state of round 5 (all centroids on the grand mean, spread 0.0).
    Reduced N and the exact fp32 path here; the preset's D, K, m and generator."""
    d = _run(["--preset", "fcm10m", "--n-per-gpu", "20000", "--dtype", "fp32", "--steps", "6",
              "--warmup", "0", "--no-steady"], timeout=900)
    assert d["config"]["D"] == 128 and d["config"]["K"] == 1024
    assert d["config"]["fuzzifier"] == 2.0 and "std 0.25" in d["data"]
    assert d["check"]["final_ws_spread"] > 0.1, d["check"]
