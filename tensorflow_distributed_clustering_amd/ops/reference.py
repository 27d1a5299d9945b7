"""Plain-PyTorch reference implementations of every hot op.

These are the numerics oracle for the HIP kernels (tests compare against them
in fp32/fp64) and the CPU execution path (gloo ranks, no GPU).  They follow the
semantics of the reference engine:

* K-Means tower: squared distances, first-minimum argmin, per-cluster sums and
  counts (`scripts/distribuitedClustering.py:221-248`; segment-sum variant
  `notebooks/visualization.ipynb:256-271`).
* FCM tower: ``d^(-2/(m-1))`` row-normalised memberships, NaN->0 guard,
  ``w = u^m``, ``W^T X`` and ``sum(W)`` (`scripts/distribuitedClustering.py:117-137`).

Everything works chunk-wise over rows so a [N, K] matrix is never materialised
for the whole shard (the reference's [N, K, D] tiles are what made every
50M+ run OOM, `scripts/executions_log.csv:2-241`).
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch

_DEF_CHUNK_ELEMS = 1 << 26  # bound on chunk_rows * K


def _chunk_rows(n: int, k: int, chunk_elems: int = _DEF_CHUNK_ELEMS) -> int:
    return max(1, min(n, chunk_elems // max(1, k)))


def pairwise_sqdist(x: torch.Tensor, c: torch.Tensor, exact: bool = False) -> torch.Tensor:
    """Squared L2 distances [n, K].

    exact=True uses the difference form sum((x-c)^2) (what the reference
    computes, `distribuitedClustering.py:228-230`); otherwise the GEMM
    expansion ||x||^2 - 2 x.c + ||c||^2 clamped at 0.
    """
    if exact:
        return ((x[:, None, :] - c[None, :, :]) ** 2).sum(-1)
    xx = (x * x).sum(1, keepdim=True)
    cc = (c * c).sum(1)[None, :]
    d = torch.addmm(cc, x, c.t(), beta=1.0, alpha=-2.0) + xx
    return d.clamp_min_(0)


def assign(x: torch.Tensor, c: torch.Tensor, exact: bool = False,
           chunk_elems: int = _DEF_CHUNK_ELEMS) -> Tuple[torch.Tensor, torch.Tensor]:
    """labels[int32 n] = argmin_k d2, mind[n] = min_k d2 (first index on ties)."""
    n, k = x.shape[0], c.shape[0]
    labels = torch.empty(n, dtype=torch.int32, device=x.device)
    mind = torch.empty(n, dtype=x.dtype, device=x.device)
    if exact:
        chunk_elems = max(1, chunk_elems // max(1, x.shape[1]))
    step = _chunk_rows(n, k, chunk_elems)
    for s in range(0, n, step):
        d = pairwise_sqdist(x[s:s + step], c, exact=exact)
        d = torch.nan_to_num(d, nan=float("inf"))  # a NaN (poisoned) centroid never wins
        v, i = d.min(1)
        labels[s:s + step] = i.to(torch.int32)
        mind[s:s + step] = v
    return labels, mind


def cluster_sums(x: torch.Tensor, labels: torch.Tensor, k: int,
                 acc_dtype: torch.dtype = torch.float64) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-cluster sum of points [K, D] and counts [K] (unsorted segment sum)."""
    sums = torch.zeros(k, x.shape[1], dtype=acc_dtype, device=x.device)
    sums.index_add_(0, labels.long(), x.to(acc_dtype))
    counts = torch.bincount(labels.long(), minlength=k)[:k].to(acc_dtype)
    return sums, counts


def finalize(sums: torch.Tensor, counts: torch.Tensor, old: torch.Tensor,
             empty_cluster: str = "keep") -> torch.Tensor:
    """new centroid = sums / counts with the configured empty-cluster policy.

    'nan' reproduces the reference: 0/0 -> NaN (`distribuitedClustering.py:262`).
    """
    cnt = counts[:, None].to(sums.dtype)
    new = sums / cnt
    empty = (counts == 0)
    if empty.any():
        if empty_cluster == "keep" or empty_cluster == "reseed":
            new[empty] = old[empty].to(new.dtype)
        elif empty_cluster == "zero":
            new[empty] = 0
        else:  # 'nan' / 'nan_any': the reference's 0/0 (`distribuitedClustering.py:262`)
            new[empty] = float("nan")
    return new.to(old.dtype)


def fcm_memberships(x: torch.Tensor, c: torch.Tensor, m: float,
                    nan_to_zero: bool = True, exact: Optional[bool] = None) -> torch.Tensor:
    """u[n, K]; u_ik = d_ik^(-2/(m-1)) / sum_k' d_ik'^(-2/(m-1)).

    nan_to_zero=True is the reference guard (`distribuitedClustering.py:125-126`):
    a point exactly on a centroid gets inf/inf = NaN -> 0 membership everywhere.
    False gives the mathematically correct one-hot membership for such points.
    """
    if m <= 1.0:
        raise ValueError(f"FCM fuzzifier must be > 1, got {m} (reference uses m := D; D=1 divides by zero)")
    if exact is None:  # difference form (the reference's) for small D; GEMM form above
        exact = x.shape[1] <= 16
    d = pairwise_sqdist(x, c, exact=exact).sqrt()
    t = d.pow(-2.0 / (m - 1.0))
    u = t / t.sum(1, keepdim=True)
    bad = torch.isnan(u)
    if bad.any():
        if nan_to_zero:
            u = torch.where(bad, torch.zeros_like(u), u)
        else:
            zero = (d == 0)
            rows = zero.any(1)
            onehot = zero.to(u.dtype) / zero.sum(1, keepdim=True).clamp_min(1).to(u.dtype)
            u = torch.where(rows[:, None], onehot, u)
    return u


def fcm_partial(x: torch.Tensor, c: torch.Tensor, m: float, nan_to_zero: bool = True,
                acc_dtype: torch.dtype = torch.float64,
                chunk_elems: int = _DEF_CHUNK_ELEMS,
                exact: Optional[bool] = None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """FCM tower: (sum_i w_ki x_i [K, D], sum_i w_ki [K], labels argmax_k u [n]).
    ``exact``: difference-form distances (default: for D <= 16, as fcm_memberships)."""
    n, k = x.shape[0], c.shape[0]
    wx = torch.zeros(k, x.shape[1], dtype=acc_dtype, device=x.device)
    ws = torch.zeros(k, dtype=acc_dtype, device=x.device)
    labels = torch.empty(n, dtype=torch.int32, device=x.device)
    ex = exact if exact is not None else x.shape[1] <= 16
    step = _chunk_rows(n, k, max(1, chunk_elems // max(1, x.shape[1] if ex else 4)))
    for s in range(0, n, step):
        xs = x[s:s + step]
        u = fcm_memberships(xs, c, m, nan_to_zero, exact=ex)
        w = u.pow(m)
        wx += (w.t().to(acc_dtype) @ xs.to(acc_dtype))
        ws += w.sum(0).to(acc_dtype)
        labels[s:s + step] = u.argmax(1).to(torch.int32)
    return wx, ws, labels


def inertia(x: torch.Tensor, c: torch.Tensor, labels: torch.Tensor) -> float:
    diff = x.double() - c.double()[labels.long()]
    return float((diff * diff).sum())


def kmeanspp(x: torch.Tensor, k: int, generator: torch.Generator,
             n_local_trials: Optional[int] = None) -> torch.Tensor:
    """Greedy k-means++ (Arthur & Vassilvitskii; sklearn's 2+log(k) trials).

    Single-shard oracle of the distributed N7 implementation.
    """
    n = x.shape[0]
    if n_local_trials is None:
        n_local_trials = 2 + int(math.log(k))
    xd = x.double()
    first = int(torch.randint(n, (1,), generator=generator).item())
    centers = [xd[first]]
    closest = ((xd - xd[first]) ** 2).sum(1)
    pot = float(closest.sum())
    for _ in range(1, k):
        if pot <= 0:
            idx = torch.randint(n, (n_local_trials,), generator=generator)
        else:
            r = torch.rand(n_local_trials, generator=generator, dtype=torch.float64) * pot
            cs = torch.cumsum(closest, 0)
            idx = torch.searchsorted(cs, r).clamp_max(n - 1)
        cand = xd[idx]
        dist = ((xd[None, :, :] - cand[:, None, :]) ** 2).sum(2)
        dist = torch.minimum(dist, closest[None, :])
        pots = dist.sum(1)
        best = int(torch.argmin(pots))
        closest = dist[best]
        pot = float(pots[best])
        centers.append(xd[int(idx[best])])
    return torch.stack(centers).to(x.dtype)
