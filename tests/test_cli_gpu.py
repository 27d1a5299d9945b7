"""GPU: the reference-compatible CLI and the segmentation app on the HIP path."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("method,extra", [("distributedKMeans", []),
                                          ("distributedFuzzyCMeans", []),
                                          ("distributedKMeans", ["--dtype", "bf16", "--graph"]),
                                          ("miniBatchKMeans", ["--batch_size", "4096"])])
def test_cli_on_gpu(gpu, tmp_path, method, extra):
    X = gaussian_blobs(60000, 5, 4, seed=3, dtype=torch.float64).numpy()
    data = tmp_path / "d.npz"
    np.savez(data, X=X, Y=np.zeros(len(X)))
    log, cen, ext = tmp_path / "l.csv", tmp_path / "c.csv", tmp_path / "e.jsonl"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "distribuitedClustering.py"),
                        "--n_obs=60000", "--n_dim=5", "--K=4", "--n_GPUs=1", "--n_max_iters=10",
                        "--seed=1", f"--log_file={log}", f"--method_name={method}",
                        f"--data_file={data}", f"--centroids_out={cen}", f"--extended_log={ext}",
                        "--log_device_placement"] + extra,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    row = open(log).read().strip().splitlines()[-1].split(",")
    assert row[0] == method and float(row[8]) > 0
    info = json.loads(open(ext).read().strip().splitlines()[-1])
    assert info["backend"].startswith("hip_"), info  # native kernels, not a torch fallback
    assert "device cuda:0" in r.stdout
    assert np.loadtxt(cen, delimiter=",").shape == (4, 5)


def test_segment_app_on_gpu(gpu):
    from tensorflow_distributed_clustering_amd.apps import segment as seg
    img, region = seg.synthetic_image(320, 320, k=6, seed=4)
    for dtype in ("fp32", "bf16"):
        s = seg.segment(img, 6, max_iter=15, dtype=dtype, device="cuda", seed=2)
        assert not s.has_nan
        purity = np.mean([np.bincount(s.labels[region == r]).max() / (region == r).sum()
                          for r in range(6)])
        assert purity > 0.97
