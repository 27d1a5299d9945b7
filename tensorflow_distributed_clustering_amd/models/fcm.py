"""Distributed Fuzzy C-Means.

Reference: ``distribuited_fuzzy_C_means`` (`scripts/distribuitedClustering.py:72-178`).
Per GPU: distances -> memberships u = d^(-2/(m-1)) / sum_k -> NaN->0 -> W = u^m ->
W X (cuBLAS DGEMM) and sum(W); CPU AddN + Div + Assign (`:139-148`).  The fuzzifier
is the data dimension (``m := M``, `:97,121,129`) -- reproduced when
``cfg.fuzzifier is None`` -- and the label pass is ``argmax_k u`` (`:141`).

Here: one fused HIP kernel per rank (N4/N5) for small K x D, one packed all-reduce of
[sum W X | sum W], and the N3 divide.
"""
from __future__ import annotations

import time
from typing import Optional

import torch

from ..config import ClusterConfig
from ..ops import make_fcm_ops
from ..parallel.dist import Comm, local_comm
from ..utils import faults
from ..utils.checkpoint import RunCheckpointer
from ..utils.timers import DeviceTimer, sync
from .init import init_centers
from .kmeans import ClusterResult, _shard_geometry


class FcmEngine:
    """Resident state of one distributed FCM run; ``step()`` = one iteration (fused tower
    kernel, one packed all-reduce of [sum W X | sum W], the N3 divide).  Timed by bench.py."""

    def __init__(self, x_local, cfg: ClusterConfig, comm: Comm, n_global: int, row_offset: int,
                 init_centers_=None, m: Optional[float] = None):
        self.cfg, self.comm = cfg, comm
        k, d = cfg.n_clusters, int(x_local.shape[1])
        self.k, self.d = k, d
        self.m = float(m) if m is not None else (float(cfg.fuzzifier) if cfg.fuzzifier is not None
                                                 else float(d))
        dev = x_local.device
        self.device = dev
        self.local = make_fcm_ops(x_local, k, cfg.dtype, self.m, cfg.fcm_nan_to_zero, cfg.backend)
        self.c0 = init_centers(cfg.init, x_local, row_offset, n_global, k, comm, cfg.seed,
                               given=init_centers_)
        self.C = self.c0.to(self.local.c_dtype).clone().contiguous()
        self.buf = torch.zeros(k * d + k, dtype=torch.float64, device=dev)
        self.wx = self.buf[: k * d].view(k, d)
        self.ws = self.buf[k * d:]
        self.labels = torch.zeros(self.local.n, dtype=torch.int32, device=dev)
        self.shift = torch.zeros(1, dtype=torch.float32, device=dev) if cfg.tol > 0 else None
        self.n_iter = 0

    def step(self):
        self.buf.zero_()
        self.local.step(self.C, self.labels, self.wx, self.ws)
        self.comm.allreduce_(self.buf)
        if self.shift is not None:
            self.shift.zero_()
        self.local.finalize(self.wx, self.ws, self.C, self.shift)
        self.n_iter += 1

    def label_pass(self):
        self.local.assign(self.C, self.labels)


class FuzzyCMeans:
    def __init__(self, cfg: ClusterConfig, comm: Optional[Comm] = None, device=None):
        self.cfg = cfg
        self.comm = comm
        self.device = device
        self.result_: Optional[ClusterResult] = None

    def fuzzifier(self, d: int) -> float:
        return float(self.cfg.fuzzifier) if self.cfg.fuzzifier is not None else float(d)

    def fit(self, x_local, init_centers_=None, n_global=None, row_offset=None) -> "FuzzyCMeans":
        cfg = self.cfg
        if cfg.spherical:
            raise ValueError("spherical=True is implemented for KMeans (Lloyd) only")
        t0 = time.perf_counter()
        x_local = torch.as_tensor(x_local)
        dev = torch.device(self.device) if self.device is not None else (
            self.comm.device if self.comm is not None else x_local.device)
        if x_local.device != dev:
            x_local = x_local.to(dev)
        if self.comm is None:
            self.comm = local_comm(dev)
        comm = self.comm
        if n_global is None or row_offset is None:
            n_global, row_offset = _shard_geometry(int(x_local.shape[0]), comm)
        k, d = cfg.n_clusters, int(x_local.shape[1])
        sync(dev)
        initialization_time = time.perf_counter() - t0

        t1 = time.perf_counter()
        ckpt = RunCheckpointer(cfg, comm, "distributedFuzzyCMeans")
        resumed = ckpt.load_for_resume(k, d)
        start_iter = 0
        if resumed is not None:
            init_centers_, start_iter = resumed.centers, resumed.n_iter
        eng = FcmEngine(x_local, cfg, comm, n_global, row_offset, init_centers_, self.fuzzifier(d))
        eng.n_iter = start_iter
        sync(dev)
        setup_time = time.perf_counter() - t1

        timer = DeviceTimer(dev)
        timer.start()
        history = []
        centers_host = lambda: eng.C.double().cpu().numpy()
        for _ in range(start_iter, cfg.max_iter):
            eng.step()
            n_iter = eng.n_iter
            if eng.shift is not None:
                sv = float(eng.shift.item())
                history.append({"iter": n_iter, "shift": sv})
                if sv <= cfg.tol:
                    break
            ckpt.maybe_save(n_iter, centers_host)
            faults.maybe_fail(str(n_iter), comm.rank)
        computation_time = timer.stop()
        n_iter = eng.n_iter
        ckpt.maybe_save(n_iter, centers_host, final=True)

        if cfg.label_pass:
            eng.label_pass()
        self.engine_ = eng
        self.result_ = ClusterResult(
            centers=eng.C.double().cpu().numpy(), init_centers=eng.c0.cpu().numpy(),
            labels=eng.labels, counts=eng.ws.double().cpu().numpy(), n_iter=n_iter, inertia=None,
            setup_time=setup_time, initialization_time=initialization_time,
            computation_time=computation_time, backend=eng.local.name, history=history,
            n_global=n_global)
        return self

    @property
    def cluster_centers_(self):
        return self.result_.centers

    def _centers_on(self, dev, dtype):
        if self.result_ is None:
            raise RuntimeError("fit() first")
        return torch.as_tensor(self.result_.centers, device=dev).to(dtype)

    def predict(self, x: torch.Tensor) -> torch.Tensor:
        """Labels (argmax membership, `distribuitedClustering.py:141`) of new points against
        the fitted centers, with the same local ops as the fit (no collectives)."""
        x = torch.as_tensor(x)
        d = int(x.shape[1])
        ops = make_fcm_ops(x, self.cfg.n_clusters, self.cfg.dtype, self.fuzzifier(d),
                           self.cfg.fcm_nan_to_zero, self.cfg.backend)
        labels = torch.empty(int(x.shape[0]), dtype=torch.int32, device=x.device)
        ops.assign(self._centers_on(x.device, ops.c_dtype), labels)
        return labels

    def memberships(self, x: torch.Tensor, chunk_rows: int = 1 << 16) -> torch.Tensor:
        """Soft memberships u [n, K] of new points (fp64 oracle formula, chunked)."""
        from ..ops import reference as ref
        x = torch.as_tensor(x)
        c = self._centers_on(x.device, torch.float64)
        m = self.fuzzifier(int(x.shape[1]))
        return torch.cat([ref.fcm_memberships(x[s:s + chunk_rows].double(), c, m,
                                              self.cfg.fcm_nan_to_zero)
                          for s in range(0, int(x.shape[0]), chunk_rows)])
