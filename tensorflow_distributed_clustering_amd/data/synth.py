"""Synthetic data generators.

* :func:`gaussian_blobs` -- the BASELINE north-star data: isotropic Gaussian blobs.
  Counter-based: every value is a pure function of ``(seed, global_row, column)``, so each
  rank generates exactly its own shard ON ITS DEVICE (no host copy, no H2D of the dataset)
  and the global dataset is identical for any world size.
* :func:`make_classification_compat` -- the reference sweep's data,
  ``sklearn.datasets.make_classification(n_samples, n_features=D, n_informative=D,
  n_redundant=0, n_classes=2, n_clusters_per_class=1, shuffle=True, random_state=seed)``
  (`scripts/new_experiment.py:9-27`), float64, saved as NPZ with keys X, Y.
"""
from __future__ import annotations

import math
import os
from typing import Tuple

import numpy as np
import torch

_M32 = 0xFFFFFFFF


def _mix32(x: torch.Tensor) -> torch.Tensor:
    # 32-bit integer finaliser evaluated in int64 (products stay < 2^59: no overflow)
    x = ((x >> 16) ^ x) * 0x45D9F3B & _M32
    x = ((x >> 16) ^ x) * 0x45D9F3B & _M32
    return (x >> 16) ^ x


def blob_centers(n_centers: int, d: int, seed: int, box: Tuple[float, float] = (-10.0, 10.0)) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return rng.uniform(box[0], box[1], size=(n_centers, d))


def _blob_rows(rows: torch.Tensor, d: int, n_centers: int, seed: int, centers: torch.Tensor,
               cluster_std: float, dtype: torch.dtype):
    """Rows with global indices ``rows`` (int64 [r, 1]) of the blob dataset, + blob ids."""
    s = int(seed) & _M32
    cols = torch.arange(d, dtype=torch.int64, device=rows.device)[None, :]
    blob = (_mix32((rows * 0x27D4EB2F + (s * 3 + 1)) & _M32) % n_centers).squeeze(1)
    h = _mix32((rows * 0x9E3779B1 + cols * 0x85EBCA6B + s) & _M32)
    u1 = (_mix32(h ^ 0x1234567).to(torch.float32) + 0.5) * (1.0 / 4294967296.0)
    u2 = (_mix32(h ^ 0x7654321).to(torch.float32) + 0.5) * (1.0 / 4294967296.0)
    del h
    z = torch.sqrt(-2.0 * torch.log(u1)) * torch.cos((2.0 * math.pi) * u2)
    del u1, u2
    z.mul_(cluster_std).add_(centers.index_select(0, blob))
    return z.to(dtype), blob


def gaussian_blobs(n_rows: int, d: int, n_centers: int, seed: int = 0, row_offset: int = 0,
                   cluster_std: float = 1.0, box: Tuple[float, float] = (-10.0, 10.0),
                   dtype: torch.dtype = torch.float32, device="cpu", chunk_rows: int = 1 << 20,
                   return_labels: bool = False):
    """Rows [row_offset, row_offset + n_rows) of the global blob dataset."""
    device = torch.device(device)
    centers = torch.as_tensor(blob_centers(n_centers, d, seed, box), dtype=torch.float32,
                              device=device)
    out = torch.empty(n_rows, d, dtype=dtype, device=device)
    lab_out = torch.empty(n_rows, dtype=torch.int32, device=device) if return_labels else None
    chunk_rows = max(1, min(chunk_rows, (1 << 27) // max(1, d)))
    for r0 in range(0, n_rows, chunk_rows):
        r1 = min(n_rows, r0 + chunk_rows)
        rows = torch.arange(row_offset + r0, row_offset + r1, dtype=torch.int64, device=device)[:, None]
        z, blob = _blob_rows(rows, d, n_centers, seed, centers, cluster_std, dtype)
        out[r0:r1] = z
        if return_labels:
            lab_out[r0:r1] = blob.to(torch.int32)
        del z
    return (out, lab_out) if return_labels else out


def gaussian_blob_rows(indices, d: int, n_centers: int, seed: int = 0, cluster_std: float = 1.0,
                       box: Tuple[float, float] = (-10.0, 10.0), dtype=torch.float64, device="cpu"):
    """Arbitrary global rows of the blob dataset (same values as :func:`gaussian_blobs`)."""
    device = torch.device(device)
    centers = torch.as_tensor(blob_centers(n_centers, d, seed, box), dtype=torch.float32, device=device)
    rows = torch.as_tensor(list(indices), dtype=torch.int64, device=device)[:, None]
    z, _ = _blob_rows(rows, d, n_centers, seed, centers, cluster_std, torch.float32)
    return z.to(dtype)


def make_classification_compat(n_obs: int, n_dim: int, seed: int):
    from sklearn.datasets import make_classification
    X, Y = make_classification(n_samples=n_obs, n_features=n_dim, n_informative=n_dim,
                               n_redundant=0, n_classes=2, n_clusters_per_class=1,
                               shuffle=True, random_state=seed)
    return X, Y


def make_data(path: str, n_obs: int, n_dim: int, seed: int, kind: str = "classification",
              n_centers: int = 2):
    """Write the NPZ the reference CLI consumes (keys X float64 [N, D], Y int)."""
    if os.path.exists(path):
        os.remove(path)  # reference deletes any old file (`scripts/new_experiment.py:11-14`)
    if kind == "classification":
        X, Y = make_classification_compat(n_obs, n_dim, seed)
    elif kind == "blobs":
        Xt, Yt = gaussian_blobs(n_obs, n_dim, n_centers, seed, dtype=torch.float64,
                                return_labels=True)
        X, Y = Xt.numpy(), Yt.numpy()
    else:
        raise ValueError(kind)
    np.savez(path, X=X, Y=Y)
    return path
