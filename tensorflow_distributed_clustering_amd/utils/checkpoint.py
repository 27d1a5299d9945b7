"""Checkpoint / resume of a clustering run (the reference had none --
centroids were never persisted, `scripts/distribuitedClustering.py:391-405`).

The state of an iterative clustering run is tiny and replicated on every rank:
centroids C[K, D], the number of completed iterations, and (mini-batch) the per-center
counts.  Rank 0 writes it as an NPZ -- arrays plus a JSON metadata string, nothing
pickled -- through a temp file + ``os.replace`` so a crash mid-write never leaves a
torn checkpoint.  Loading uses ``allow_pickle=False``.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import Dict, Optional

import numpy as np

FORMAT = "tdc-checkpoint-v1"


@dataclass
class Checkpoint:
    method: str
    n_iter: int
    centers: np.ndarray                 # [K, D] float64
    meta: dict = field(default_factory=dict)
    arrays: Dict[str, np.ndarray] = field(default_factory=dict)


def save(path: str, ckpt: Checkpoint) -> None:
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    meta = dict(ckpt.meta, format=FORMAT, method=ckpt.method, n_iter=int(ckpt.n_iter))
    payload = {"centers": np.asarray(ckpt.centers, dtype=np.float64),
               "meta_json": np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)}
    for k, v in ckpt.arrays.items():
        payload["arr_" + k] = np.asarray(v)
    tmp = f"{path}.tmp.{os.getpid()}"
    with open(tmp, "wb") as f:
        np.savez(f, **payload)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


def load(path: str) -> Checkpoint:
    with np.load(path, allow_pickle=False) as z:
        meta = json.loads(bytes(z["meta_json"]).decode())
        if meta.get("format") != FORMAT:
            raise ValueError(f"{path}: not a {FORMAT} file")
        arrays = {k[4:]: z[k] for k in z.files if k.startswith("arr_")}
        return Checkpoint(method=meta["method"], n_iter=int(meta["n_iter"]),
                          centers=np.array(z["centers"]), meta=meta, arrays=arrays)


class RunCheckpointer:
    """Per-run hook used by the model drivers: resume lookup + periodic saves."""

    def __init__(self, cfg, comm, method: str):
        self.path = cfg.checkpoint_path
        self.every = int(cfg.checkpoint_every)
        self.resume = bool(cfg.resume)
        self.comm = comm
        self.method = method
        self.cfg = cfg

    @property
    def enabled(self) -> bool:
        return bool(self.path)

    def load_for_resume(self, k: int, d: int) -> Optional[Checkpoint]:
        if not (self.path and self.resume and os.path.exists(self.path)):
            return None
        ck = load(self.path)
        if ck.method != self.method or ck.centers.shape != (k, d):
            raise ValueError(f"checkpoint {self.path} is for {ck.method} {ck.centers.shape}, "
                             f"not {self.method} ({k}, {d})")
        return ck

    def due(self, n_iter: int) -> bool:
        """Would maybe_save(n_iter) write a periodic checkpoint?"""
        return bool(self.path) and self.every > 0 and n_iter % self.every == 0

    def maybe_save(self, n_iter: int, centers_fn, arrays_fn=None, final: bool = False) -> bool:
        if not self.path:
            return False
        if not final and (self.every <= 0 or n_iter % self.every != 0):
            return False
        centers = centers_fn()              # every rank participates in any device sync
        arrays = arrays_fn() if arrays_fn else {}
        if self.comm.is_root:
            save(self.path, Checkpoint(self.method, n_iter, centers,
                                       meta={"config": self.cfg.to_dict(),
                                             "world_size": self.comm.world_size},
                                       arrays=arrays))
        return True
