"""Image colour segmentation (reference `notebooks/Testing Images.ipynb`).

The notebook flattened an RGB image to pixels [H*W, 3] float64 (`:289-306,319,329`),
clustered the colours with its TF K-Means, rebuilt the segmented image as
``center[labels]`` (`:425-434`), timed every frame, cross-checked the centers against
``cv2.kmeans(K, criteria=(EPS+MAX_ITER, 10, 1.0), attempts=10, KMEANS_RANDOM_CENTERS)``
(`:344-347,359-368`) and flagged NaN centers from empty clusters (`:450-462`).

OpenCV is not part of this stack; :func:`cv_style_kmeans` is a NumPy implementation of the
same baseline (best of ``attempts`` Lloyd runs from uniform random centers in the data's
bounding box, stopping at ``max_iter`` or a center move <= ``eps``), used as the
cross-check oracle.

    python -m tensorflow_distributed_clustering_amd.apps.segment --image in.png --K 8 \\
        --out seg.png [--compare] [--dtype fp32] [--device cuda]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np
import torch

from ..config import ClusterConfig
from ..models.fcm import FuzzyCMeans
from ..models.kmeans import KMeans


def load_image(path: str) -> np.ndarray:
    """RGB uint8 [H, W, 3] (PIL)."""
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("RGB"))


def save_image(path: str, img: np.ndarray) -> None:
    from PIL import Image
    Image.fromarray(np.asarray(img, dtype=np.uint8)).save(path)


def to_pixels(img: np.ndarray) -> np.ndarray:
    """[H, W, 3] -> [H*W, 3] float64 (the notebook's ``reshape((-1, 3)).astype(float64)``)."""
    return np.asarray(img, dtype=np.float64).reshape(-1, img.shape[-1])


def has_nan_centers(centers) -> bool:
    """The notebook's empty-cluster NaN detector (`Testing Images.ipynb:450-462`)."""
    return bool(np.isnan(np.asarray(centers, dtype=np.float64)).any())


def synthetic_image(h: int = 640, w: int = 640, k: int = 6, seed: int = 0,
                    noise: float = 6.0) -> Tuple[np.ndarray, np.ndarray]:
    """Test image: k flat-colour Voronoi regions + Gaussian noise; returns (img, region id)."""
    rng = np.random.default_rng(seed)
    colours = rng.uniform(20, 235, size=(k, 3))
    seeds = rng.uniform(0, 1, size=(k, 2)) * [h, w]
    yy, xx = np.mgrid[0:h, 0:w]
    d = (yy[..., None] - seeds[:, 0]) ** 2 + (xx[..., None] - seeds[:, 1]) ** 2
    region = d.argmin(-1)
    img = colours[region] + rng.normal(0, noise, size=(h, w, 3))
    return np.clip(img, 0, 255).astype(np.uint8), region


def cv_style_kmeans(pixels: np.ndarray, k: int, attempts: int = 10, max_iter: int = 10,
                    eps: float = 1.0, seed: int = 0):
    """NumPy stand-in for ``cv2.kmeans(..., KMEANS_RANDOM_CENTERS)``: (compactness, labels,
    centers) of the best attempt."""
    rng = np.random.default_rng(seed)
    x = np.asarray(pixels, dtype=np.float64)
    lo, hi = x.min(0), x.max(0)
    best = None
    xn = (x * x).sum(1)
    for _ in range(attempts):
        c = rng.uniform(lo, hi, size=(k, x.shape[1]))
        for _ in range(max_iter):
            d2 = xn[:, None] - 2 * x @ c.T + (c * c).sum(1)[None]
            lab = d2.argmin(1)
            new = c.copy()
            for j in range(k):
                m = lab == j
                if m.any():
                    new[j] = x[m].mean(0)
            move = np.sqrt(((new - c) ** 2).sum(1)).max()
            c = new
            if move <= eps:
                break
        d2 = xn[:, None] - 2 * x @ c.T + (c * c).sum(1)[None]
        lab = d2.argmin(1)
        comp = float(np.maximum(d2[np.arange(len(x)), lab], 0).sum())
        if best is None or comp < best[0]:
            best = (comp, lab, c)
    return best


@dataclass
class Segmentation:
    image: np.ndarray          # segmented [H, W, 3] uint8
    labels: np.ndarray         # [H, W] int
    centers: np.ndarray        # [K, 3] float64
    inertia: float
    seconds: float
    has_nan: bool


def segment(img: np.ndarray, k: int, max_iter: int = 20, dtype: str = "fp32",
            init: str = "kmeans++", seed: int = 0, device: Optional[str] = None,
            tol: float = 0.0, method: str = "kmeans", fuzzifier: Optional[float] = None) -> Segmentation:
    """Segment one frame.  method 'fcm' runs Fuzzy C-Means (hard labels = argmax membership;
    the notebook's FCM used m = D = 3 for RGB)."""
    h, w = img.shape[:2]
    dev = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    px = torch.from_numpy(to_pixels(img)).to(dev)
    cfg = ClusterConfig(n_clusters=k, max_iter=max_iter, dtype=dtype, init=init, seed=seed,
                        tol=tol, fuzzifier=fuzzifier)
    t0 = time.perf_counter()
    model = FuzzyCMeans if method == "fcm" else KMeans
    km = model(cfg, device=dev).fit(px)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    secs = time.perf_counter() - t0
    r = km.result_
    lab = r.labels.long().cpu().numpy()
    seg = np.clip(np.rint(np.nan_to_num(r.centers)[lab]), 0, 255).astype(np.uint8).reshape(h, w, -1)
    inertia = r.inertia
    if inertia is None:  # FCM: report the hard-assignment SSE
        inertia = float(((to_pixels(img) - r.centers[lab]) ** 2).sum())
    return Segmentation(seg, lab.reshape(h, w), r.centers, float(inertia), secs,
                        has_nan_centers(r.centers))


def benchmark_frames(n_frames: int = 10, h: int = 640, w: int = 640, k: int = 3,
                     max_iter: int = 20, dtype: str = "fp64", method: str = "kmeans",
                     device: Optional[str] = None) -> dict:
    """The notebook's per-frame protocol (`Testing Images.ipynb`): 409,600-px RGB frames,
    K=3, 20 iterations, fp64; mean seconds per frame (fit incl. setup; first frame =
    warm-up, excluded)."""
    times = []
    for f in range(n_frames + 1):
        img, _ = synthetic_image(h, w, k=max(k, 3), seed=100 + f)
        s = segment(img, k, max_iter, dtype, "random", seed=f, device=device, method=method)
        if f:
            times.append(s.seconds)
    return {"frames": n_frames, "pixels": h * w, "K": k, "iters": max_iter, "dtype": dtype,
            "method": method, "mean_seconds_per_frame": float(np.mean(times)),
            "points_iter_per_sec": h * w * max_iter / float(np.mean(times))}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="K-Means colour segmentation of an image")
    ap.add_argument("--image", help="input image (omit: synthetic 640x640 test image)")
    ap.add_argument("--K", type=int, default=8)
    ap.add_argument("--n_max_iters", type=int, default=20)
    ap.add_argument("--dtype", default="fp32", choices=["fp64", "fp32", "bf16"])
    ap.add_argument("--init", default="kmeans++", choices=["kmeans++", "random", "first_k"])
    ap.add_argument("--device", default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=None, help="write the segmented image here")
    ap.add_argument("--compare", action="store_true",
                    help="cross-check against the cv2.kmeans-style best-of-10 baseline")
    ap.add_argument("--method", default="kmeans", choices=["kmeans", "fcm"])
    ap.add_argument("--bench_frames", type=int, default=0,
                    help="run the notebook's per-frame benchmark on N synthetic 640x640 frames")
    a = ap.parse_args(argv)
    if a.bench_frames:
        print(json.dumps(benchmark_frames(a.bench_frames, k=a.K, max_iter=a.n_max_iters,
                                          dtype=a.dtype, method=a.method, device=a.device)))
        return 0
    img = load_image(a.image) if a.image else synthetic_image(seed=a.seed)[0]
    s = segment(img, a.K, a.n_max_iters, a.dtype, a.init, a.seed, a.device, method=a.method)
    out = {"pixels": int(img.shape[0] * img.shape[1]), "K": a.K, "seconds": s.seconds,
           "inertia": s.inertia, "nan_centers": s.has_nan}
    if a.compare:
        t0 = time.perf_counter()
        comp, _, _ = cv_style_kmeans(to_pixels(img), a.K, seed=a.seed)
        out.update(baseline_seconds=time.perf_counter() - t0, baseline_compactness=comp,
                   inertia_vs_baseline=s.inertia / comp if comp > 0 else None)
    if a.out:
        save_image(a.out, s.image)
    print(json.dumps(out))
    return 1 if s.has_nan else 0


if __name__ == "__main__":
    sys.exit(main())
