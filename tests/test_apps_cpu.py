"""Image segmentation app + validation plots + placement logging (reference notebooks
`Testing Images.ipynb`, `visualization.ipynb`)."""
import json
import os
import subprocess
import sys

import numpy as np
import torch

from tensorflow_distributed_clustering_amd.apps import segment as seg
from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
from tensorflow_distributed_clustering_amd.utils.plots import scatter_svg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_synthetic_segmentation_recovers_regions():
    img, region = seg.synthetic_image(160, 120, k=5, seed=3)
    s = seg.segment(img, 5, max_iter=15, dtype="fp64", device="cpu", seed=1)
    assert s.image.shape == img.shape and not s.has_nan
    # every true region maps to (almost) one label
    purity = np.mean([np.bincount(s.labels[region == r]).max() / (region == r).sum()
                      for r in range(5)])
    assert purity > 0.98
    comp, _, _ = seg.cv_style_kmeans(seg.to_pixels(img), 5, seed=0)
    assert s.inertia <= 1.01 * comp


def test_nan_detector():
    assert seg.has_nan_centers([[1.0, np.nan]]) and not seg.has_nan_centers([[1.0, 2.0]])


def test_segment_cli_roundtrip(tmp_path):
    img, _ = seg.synthetic_image(64, 80, k=4, seed=2)
    src, out = tmp_path / "in.png", tmp_path / "out.png"
    seg.save_image(str(src), img)
    r = subprocess.run([sys.executable, "-m", "tensorflow_distributed_clustering_amd.apps.segment",
                        "--image", str(src), "--K", "4", "--out", str(out), "--compare",
                        "--device", "cpu", "--dtype", "fp64"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr
    info = json.loads(r.stdout.strip().splitlines()[-1])
    assert info["pixels"] == 64 * 80 and info["inertia_vs_baseline"] <= 1.01
    assert seg.load_image(str(out)).shape == (64, 80, 3)


def test_scatter_svg(tmp_path):
    x = np.random.default_rng(0).normal(size=(500, 2))
    p = scatter_svg(str(tmp_path / "s.svg"), x, np.arange(500) % 3, x[:3], x[3:6])
    txt = open(p).read()
    assert txt.startswith("<svg") and txt.count("<circle") == 500 and txt.count("<rect") == 7


def test_cli_placement_and_plot(tmp_path):
    data = tmp_path / "d.npz"
    X = gaussian_blobs(2000, 2, 3, seed=1, dtype=torch.float64).numpy()
    np.savez(data, X=X, Y=np.zeros(2000))
    svg = tmp_path / "p.svg"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "distribuitedClustering.py"),
                        "--n_obs=2000", "--n_dim=2", "--K=3", "--n_GPUs=1", "--n_max_iters=5",
                        "--seed=1", f"--log_file={tmp_path / 'l.csv'}",
                        "--method_name=distributedKMeans", f"--data_file={data}", "--device=cpu",
                        "--log_device_placement", f"--plot_out={svg}"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "[placement] rank 0/1" in r.stdout and "rows [0, 2000)" in r.stdout
    assert svg.exists()


def test_fcm_segmentation_and_frame_bench():
    img, region = seg.synthetic_image(96, 96, k=3, seed=5)
    s = seg.segment(img, 3, max_iter=10, dtype="fp64", device="cpu", method="fcm", seed=1)
    assert s.image.shape == img.shape and s.inertia > 0
    b = seg.benchmark_frames(n_frames=1, h=64, w=64, k=3, max_iter=3, device="cpu")
    assert b["pixels"] == 4096 and b["mean_seconds_per_frame"] > 0
