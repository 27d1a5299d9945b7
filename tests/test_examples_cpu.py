"""The examples/ scripts (reference notebook workflows) run end to end at tiny sizes."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(script, args, cwd):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", script)] + args,
                       capture_output=True, text=True, timeout=600, cwd=cwd)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


def test_batched_kmeans_2d(tmp_path):
    out = _run("batched_kmeans_2d.py", ["--n", "40000", "--k", "4", "--iters", "5"], tmp_path)
    assert out["kmeans"]["n_iter"] == 5 and out["fcm"]["n_iter"] == 5
    assert (tmp_path / "batched_2d_kmeans.svg").exists() and (tmp_path / "batched_2d_fcm.svg").exists()


def test_segment_sum_variant(tmp_path):
    out = _run("segment_sum_variant.py", ["--n", "20000", "--k", "4", "--iters", "8"], tmp_path)
    assert out["kmeans_inertia"] > 0 and len(out["fcm_centers"]) == 4


def test_out_of_core_npz(tmp_path):
    x = np.random.default_rng(0).normal(size=(20000, 6))
    np.savez(tmp_path / "d.npz", X=x, Y=np.zeros(20000))
    out = _run("out_of_core_npz.py", ["--data", str(tmp_path / "d.npz"), "--k", "5",
                                       "--dtype", "fp64", "--chunk_rows", "3000"], tmp_path)
    assert out["n"] == 20000 and out["streamed"] and out["n_iter"] == 10


def test_online_serving(tmp_path):
    out = _run("online_serving.py", ["--d", "8", "--k", "6", "--batches", "5", "--batch", "2000",
                                     "--requests", "4", "--request_rows", "256"], tmp_path)
    assert out["batches_seen"] == 5 and out["label_agreement"] > 0.999
