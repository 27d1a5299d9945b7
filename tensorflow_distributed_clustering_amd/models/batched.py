"""Reference batch-averaging mode (opt-in): cluster N batches independently, average.

The reference CLI splits the dataset with ``np.array_split(X, num_batches)``, runs the
whole algorithm on each batch separately, *sums* the setup / initialization /
computation times and returns ``np.mean`` of the per-batch centers without aligning
them (`scripts/distribuitedClustering.py:296-318`, batches made at `:335`; the notebook
variant is `notebooks/New-Distributed-KMeans.ipynb:225-312`).  It starts at one batch and
doubles the count on an out-of-memory error (`:328-360`).

This framework does not need batches for memory (the resident path holds 288 GB of
rows per GPU and :mod:`..data.stream` runs an exact streamed Lloyd beyond that), so the
default CLI path is one exact fit.  :func:`fit_batches_averaged` reproduces the
reference's batched *semantics* for users who want its numbers: global batch ``b`` is
``array_split`` of the global rows, and each batch is sharded over all ranks with the
same ``array_split`` rule (`:array_split` per batch, then per GPU), so every rank
works on every batch as in the reference's in-graph replication.
"""
from __future__ import annotations

import dataclasses
import os
from typing import Callable, Optional

import numpy as np
import torch

from ..parallel.dist import local_comm, shard_bounds
from .kmeans import ClusterResult


def batch_checkpoint_path(path: str, b: int) -> str:
    """Checkpoint file of batch ``b`` (``run.npz`` -> ``run_b1.npz``): every batch resumes
    from its own state; the base path receives the averaged centers at the end."""
    if not path:
        return path
    root, ext = os.path.splitext(path)
    return f"{root}_b{b}{ext}"


def _shared_init(model, x_batch0: torch.Tensor, row_offset: int, n_batch0: int) -> np.ndarray:
    """ONE set of initial centers for every batch, as the reference does: it builds
    ``initial_centers = X[0:K]`` once (`distribuitedClustering.py:325`) and passes the same
    array to each batch fit, which keeps cluster identities aligned before ``np.mean``.
    Computed collectively with the model's configured init on batch 0's rows (``first_k``
    gives exactly the reference's global ``X[0:K]``)."""
    from .init import init_centers
    cfg = model.cfg
    comm = model.comm if model.comm is not None else local_comm(x_batch0.device)
    dev = comm.device
    method = cfg.init if cfg.init != "given" else "first_k"
    c = init_centers(method, x_batch0.to(dev), row_offset, n_batch0, cfg.n_clusters, comm,
                     cfg.seed, kpp_max_k=cfg.kpp_max_k, kpp_sample_per_k=cfg.kpp_sample_per_k,
                     kpp_sample_min=cfg.kpp_sample_min)
    return c.double().cpu().numpy()


def batch_bounds(n_global: int, num_batches: int, b: int):
    """Global row range [s, e) of batch ``b`` (``np.array_split`` rule)."""
    return shard_bounds(n_global, num_batches, b)


def fit_batches_averaged(make_model: Callable[[], object], rows, n_global: int,
                         num_batches: int, rank: int, world: int,
                         init_centers_: Optional[np.ndarray] = None) -> ClusterResult:
    """Fit ``num_batches`` independent models from one shared start and average their
    centers.

    ``rows`` is indexable by global row (an ``np.memmap`` of the NPZ member or any
    array); this rank copies only its share of each batch.  ``make_model()`` returns a
    fresh :class:`KMeans` / :class:`FuzzyCMeans` bound to the job's communicator.
    Phase times are summed over batches and ``n_iter`` is the largest batch count, as
    the reference reports them.
    """
    if num_batches < 1:
        raise ValueError("num_batches must be >= 1")
    if num_batches > n_global:
        raise ValueError(f"num_batches={num_batches} exceeds the {n_global} rows")
    centers, results = [], []
    base_ckpt = ""
    for b in range(num_batches):
        bs, be = batch_bounds(n_global, num_batches, b)
        s, e = shard_bounds(be - bs, world, rank)
        x = torch.from_numpy(np.array(rows[bs + s: bs + e], copy=True))
        model = make_model()
        base_ckpt = model.cfg.checkpoint_path
        if base_ckpt:
            model.cfg = dataclasses.replace(model.cfg,
                                            checkpoint_path=batch_checkpoint_path(base_ckpt, b))
        if init_centers_ is None:
            init_centers_ = _shared_init(model, x, s, be - bs)
        model.fit(x, init_centers_=init_centers_, n_global=be - bs, row_offset=s)
        r = model.result_
        results.append(r)
        centers.append(np.asarray(r.centers, dtype=np.float64))
        del model, x
    first = results[0]
    avg = np.mean(np.stack(centers), axis=0)
    if base_ckpt and rank == 0:
        from ..utils.checkpoint import Checkpoint, save
        save(base_ckpt, Checkpoint("batched-average", max(r.n_iter for r in results), avg,
                                   meta={"num_batches": num_batches,
                                         "batch_checkpoints": [batch_checkpoint_path(base_ckpt, b)
                                                               for b in range(num_batches)]}))
    return ClusterResult(
        centers=avg,
        init_centers=first.init_centers,
        labels=None,  # per-batch labels refer to different center sets
        counts=None,
        n_iter=max(r.n_iter for r in results),
        inertia=None,
        setup_time=sum(r.setup_time for r in results),
        initialization_time=sum(r.initialization_time for r in results),
        computation_time=sum(r.computation_time for r in results),
        backend=first.backend,
        history=[{"batch": i, "n_iter": r.n_iter, "inertia": r.inertia}
                 for i, r in enumerate(results)],
        n_global=n_global,
        streamed=any(r.streamed for r in results),
    )
