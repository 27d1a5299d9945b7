"""Distributed Fuzzy C-Means.

Reference: ``distribuited_fuzzy_C_means`` (`scripts/distribuitedClustering.py:72-178`).
Per GPU: distances -> memberships u = d^(-2/(m-1)) / sum_k -> NaN->0 -> W = u^m ->
W X (cuBLAS DGEMM) and sum(W); CPU AddN + Div + Assign (`:139-148`).  The fuzzifier
is the data dimension (``m := M``, `:97,121,129`) -- reproduced when
``cfg.fuzzifier is None`` -- and the label pass is ``argmax_k u`` (`:141`).

Here: the native FCM tower per rank (``ops.make_fcm_ops``: fused small-K*D kernel, exact
SIMT tower, or the bf16x3 MFMA tower), one packed all-reduce of [sum W X | sum W], the N3
divide.  Like K-Means, the shard may stay on the host and stream through HBM in chunks
(the partials of all chunks add up before the single all-reduce, so a streamed pass is the
exact FCM step), and an out-of-memory error -- while building the engine or inside any
iteration, on any rank -- makes every rank continue streamed with smaller chunks (the
reference doubled its batch count and restarted on ResourceExhaustedError, `:331-360`).
"""
from __future__ import annotations

import math
import time
import weakref
from typing import Optional

import numpy as np
import torch

from ..config import ClusterConfig
from ..data.stream import HostSource, ResidentSource, plan_chunk_rows, plan_resident_rows
from ..ops import make_fcm_ops
from ..parallel.dist import Comm, local_comm
from ..utils import faults
from ..utils.checkpoint import RunCheckpointer
from ..utils.timers import DeviceTimer, sync
from .init import init_centers, init_centers_from_source
from .kmeans import (ClusterResult, OomGuard, _release, _retry_chunk, _shard_geometry,
                     build_engine_collective)


# log2 of the smallest typical weight w = u^m (u ~ 1/K) that fp32 carries with headroom
# (smallest normal fp32: 2^-126)
FCM_FP32_MIN_LOG2_W = -100.0


def fcm_dtype(cfg: ClusterConfig, m: Optional[float] = None) -> torch.dtype:
    """Row / membership dtype: fp32 for fp32 and bf16/fp8 configs (bf16 selects the MFMA
    towers, whose distances are bf16x3 -- 16 mantissa bits per operand -- and whose W^T X
    weights are bf16; fp32 from K = 64, D = 64 is promoted to the fp64 matrix-core path).

    With the reference's fuzzifier m = D (`distribuitedClustering.py:121,129`) the weights
    u^m of a point's typical memberships u ~ 1/K fall to K^-m: 2^-144 at K=64, D=24, below
    fp32's range, where every sum over them flushes to zero and the centroids become 0/0.
    The reference ran fp64 throughout; such configurations are promoted to fp64 here."""
    if cfg.dtype == "fp64":
        return torch.float64
    if m is not None and -m * math.log2(max(2, cfg.n_clusters)) < FCM_FP32_MIN_LOG2_W:
        return torch.float64
    return torch.float32


class FcmEngine(OomGuard):
    """Resident or streamed state of one distributed FCM run; ``step()`` = one iteration
    (native tower over the shard or its chunks, one packed all-reduce of
    [sum W X | sum W | oom flag], the N3 divide).  Timed by bench.py."""

    def __init__(self, source, cfg: ClusterConfig, comm: Comm, n_global: int, row_offset: int,
                 init_centers_=None, m: Optional[float] = None, chunk_rows: int = 0,
                 defer_init: bool = False):
        self.cfg, self.comm = cfg, comm
        self.n_global, self.row_offset = n_global, row_offset
        k = cfg.n_clusters
        if isinstance(source, torch.Tensor):
            d = int(source.shape[1])
            dev = source.device
            self._x0 = source
            self.n_local = int(source.shape[0])
        else:
            d = int(source.d)
            dev = torch.device(getattr(source, "device", comm.device))
            self._x0 = None
            self.n_local = int(source.n_rows)
        self.k, self.d, self.device = k, d, dev
        self.m = float(m) if m is not None else (float(cfg.fuzzifier) if cfg.fuzzifier is not None
                                                 else float(d))
        tdt = fcm_dtype(cfg, self.m)
        # bf16 / fp8: the MFMA towers (fp32 memberships, bf16x3 distances, bf16 weights);
        # fp32: the exact difference-form towers
        dt_name = ("fp64" if tdt == torch.float64 else
                   "bf16" if cfg.dtype in ("bf16", "fp8") else "fp32")
        self.dtype_name = dt_name
        if tdt == torch.float64 and cfg.dtype != "fp64" and comm.is_root:
            print(f"[fcm] fuzzifier m={self.m:g} with K={k}: weights u^m ~ K^-m underflow fp32; "
                  f"computing in fp64", flush=True)
        if isinstance(source, torch.Tensor) and not chunk_rows:
            self.local = make_fcm_ops(source, k, dt_name, self.m, cfg.fcm_nan_to_zero, cfg.backend,
                                      cfg.fcm_distances)
            self.source = None
        else:
            if isinstance(source, torch.Tensor):  # device-resident shard, walked in chunks
                source = ResidentSource(source.to(tdt), (tdt, d), row_offset)
            probe = torch.zeros(1, d, dtype=tdt, device=dev)
            self.local = make_fcm_ops(probe, k, dt_name, self.m, cfg.fcm_nan_to_zero, cfg.backend,
                                      cfg.fcm_distances)
            self.source = source
        self.chunk_rows = chunk_rows
        self.streamed = self.source is not None
        self._init_given = init_centers_
        # [sum W X | sum W | oom flag] (fp64)
        self.oom_guard = bool(cfg.oom_recovery)
        self.buf = torch.zeros(k * d + k + (1 if self.oom_guard else 0), dtype=torch.float64,
                               device=dev)
        self.wx = self.buf[: k * d].view(k, d)
        self.ws = self.buf[k * d: k * d + k]
        self.oom_flag = self.buf[-1:] if self.oom_guard else None
        self.C = torch.zeros(k, d, dtype=self.local.c_dtype, device=dev)
        self.labels = torch.zeros(self.n_local, dtype=torch.int32, device=dev)
        if hasattr(self.local, "skip_step_labels"):
            self.local.skip_step_labels = bool(cfg.label_pass)  # the final pass writes them
        self.shift = torch.zeros(1, dtype=torch.float32, device=dev) if cfg.tol > 0 else None
        self.n_iter = 0
        self.c0 = None
        if self.oom_guard:
            self._oom_alloc()
        if not defer_init:
            self.init_centroids()

    def init_centroids(self):
        cfg = self.cfg
        if self._x0 is not None:
            c0 = init_centers(cfg.init, self._x0, self.row_offset, self.n_global, self.k,
                              self.comm, cfg.seed, given=self._init_given,
                              kpp_max_k=cfg.kpp_max_k, kpp_sample_per_k=cfg.kpp_sample_per_k,
                              kpp_sample_min=cfg.kpp_sample_min)
        else:
            c0 = init_centers_from_source(cfg.init, self.source, self.row_offset, self.n_global,
                                          self.k, self.comm, cfg.seed, given=self._init_given,
                                          d=self.d, kpp_max_k=cfg.kpp_max_k,
                                          kpp_sample_per_k=cfg.kpp_sample_per_k,
                                          kpp_sample_min=cfg.kpp_sample_min)
        self.c0 = c0
        self.C.copy_(c0.to(self.local.c_dtype))
        self._x0 = None
        return self

    def _chunks(self):
        return self.source.chunks(self.chunk_rows)

    def _local_step(self):
        if not self.streamed:
            self.local.step(self.C, self.labels, self.wx, self.ws)
            return
        for start, chunk in self._chunks():
            s = start - self.row_offset
            self.local.bind(chunk).step(self.C, self.labels[s:s + chunk.shape[0]], self.wx,
                                        self.ws)
        self.local.unbind()

    def step(self):
        self.buf.zero_()
        try:
            if self.oom_guard and not self._warming:
                faults.maybe_fail(str(self.n_iter + 1), self.comm.rank, kinds=("oom",))
            self._local_step()
        except Exception as e:  # noqa: BLE001 - filtered right below
            if self.oom_flag is None or not faults.is_oom(e):
                raise
            self.buf.zero_()
            self.oom_flag.fill_(1.0)  # every rank still joins the all-reduce and sees it
        self.comm.allreduce_(self.buf)
        if self.shift is not None:
            self.shift.zero_()
        self.local.finalize(self.wx, self.ws, self.C, self.shift)
        self.n_iter += 1

    rsag = False  # (OomGuard) the FCM partials always go through one all-reduce

    def snapshot(self) -> dict:
        """Restart state (bench.py: timed iterations 1..K from the init); see LloydEngine."""
        return {"C": self.C.clone(), "n_iter": self.n_iter}

    def rewind(self, snap: dict):
        self.C.copy_(snap["C"])
        self.local.prepare(self.C)
        self.n_iter = snap["n_iter"]

    def centers(self) -> torch.Tensor:
        return self.C

    def label_pass(self):
        if not self.streamed:
            self.local.assign(self.C, self.labels)
            return
        for start, chunk in self._chunks():
            s = start - self.row_offset
            self.local.bind(chunk).assign(self.C, self.labels[s:s + chunk.shape[0]])
        self.local.unbind()


class FuzzyCMeans:
    def __init__(self, cfg: ClusterConfig, comm: Optional[Comm] = None, device=None):
        self.cfg = cfg
        self.comm = comm
        self.device = device
        self.result_: Optional[ClusterResult] = None

    def fuzzifier(self, d: int) -> float:
        return float(self.cfg.fuzzifier) if self.cfg.fuzzifier is not None else float(d)

    def _target_device(self, x):
        if self.device is not None:
            return torch.device(self.device)
        if self.comm is not None:
            return self.comm.device
        if isinstance(x, torch.Tensor):
            return x.device
        return torch.device(getattr(x, "device", "cpu"))

    def _make_source(self, x_local, dev, row_offset, chunk_override: int = 0):
        """(source, chunk_rows): the resident shard, or a host source streamed in chunks
        (native RowStreamer, pinned ring, copy stream; fp32 or fp64 rows) when it does not
        fit the HBM budget (or cfg.chunk_rows / an OOM retry asks)."""
        cfg = self.cfg
        want = chunk_override or cfg.chunk_rows
        if hasattr(x_local, "chunks"):
            return x_local, want or (1 << 22)
        tdt = fcm_dtype(cfg, self.fuzzifier(int(x_local.d if hasattr(x_local, "d")
                                                else x_local.shape[1])))
        if isinstance(x_local, torch.Tensor) and x_local.device.type != "cpu":
            return x_local.to(dev), want
        xn = x_local.numpy() if isinstance(x_local, torch.Tensor) else np.asarray(x_local)
        n, d = xn.shape
        layout = (tdt, d)
        if dev.type == "cuda":
            es = 8 if tdt == torch.float64 else 4
            # MFMA tower keeps hi/lo bf16 rows + norms + row info next to the chunk
            row_bytes = d * es + 4 * d + 16
            # the wide towers (D > 128) hold a [rows, K] block of up to 2^28 elements; the
            # fused fp64 path (ops.fcm_f64_mfma) an fp64 one, and fp32 rows promoted
            from ..ops import HipWideFCM, fcm_f64_mfma
            if cfg.dtype not in ("bf16", "fp8") and fcm_f64_mfma(
                    cfg.n_clusters, d, "fp64" if es == 8 else "fp32"):
                g_bytes = HipWideFCM.chunk_elems * 8
                row_bytes += 8 * d + 8 if es == 4 else 8
            else:
                g_bytes = HipWideFCM.chunk_elems * es if d > 128 else 0
            chunk = want or plan_chunk_rows(n, row_bytes, cfg.n_clusters, d, dev,
                                            cfg.hbm_budget_gb, extra_fixed=g_bytes)
            if chunk:
                resident = 0 if want else plan_resident_rows(n, row_bytes, chunk, cfg.n_clusters,
                                                             d, dev, cfg.hbm_budget_gb,
                                                             extra_fixed=g_bytes)
                return HostSource(xn, layout, dev, row_offset, resident_rows=resident), chunk
        elif want:
            return HostSource(xn, layout, dev, row_offset), want
        return torch.as_tensor(xn).to(dev), want

    def _build_engine(self, x_local, dev, comm, n_global, row_offset, n_local, init_c,
                      start_iter, m, chunk: int = 0):
        """FcmEngine under the collective OOM agreement (see KMeans._build_engine)."""
        cfg = self.cfg
        return build_engine_collective(
            "fcm", cfg, comm, dev, n_local, start_iter, chunk,
            lambda c: self._make_source(x_local, dev, row_offset, c),
            lambda source, chunk_rows: FcmEngine(source, cfg, comm, n_global, row_offset, init_c,
                                                 m, chunk_rows, defer_init=True))

    def fit(self, x_local, init_centers_=None, n_global=None, row_offset=None) -> "FuzzyCMeans":
        cfg = self.cfg
        if cfg.spherical:
            raise ValueError("spherical=True is implemented for KMeans (Lloyd) only")
        t0 = time.perf_counter()
        if not hasattr(x_local, "chunks") and not isinstance(x_local, (torch.Tensor, np.ndarray)):
            x_local = np.asarray(x_local)
        dev = self._target_device(x_local)
        if self.comm is None:
            self.comm = local_comm(dev)
        comm = self.comm
        n_local = int(x_local.n_rows if hasattr(x_local, "n_rows") else x_local.shape[0])
        d = int(x_local.d if hasattr(x_local, "d") else x_local.shape[1])
        if n_global is None or row_offset is None:
            n_global, row_offset = _shard_geometry(n_local, comm)
        ckpt = RunCheckpointer(cfg, comm, "distributedFuzzyCMeans")
        resumed = ckpt.load_for_resume(cfg.n_clusters, d)
        start_iter = 0
        if resumed is not None:
            init_centers_, start_iter = resumed.centers, resumed.n_iter
        m = self.fuzzifier(d)
        eng, initialization_time = self._build_engine(x_local, dev, comm, n_global, row_offset,
                                                      n_local, init_centers_, start_iter, m)
        self.engine_ = eng
        if cfg.warmup and cfg.max_iter > eng.n_iter:
            eng.warmup()
        sync(dev)
        setup_time = time.perf_counter() - t0 - initialization_time

        self._retired = []  # weak references to engines replaced after an OOM
        timer = DeviceTimer(dev)
        timer.start()
        history = []
        centers_host = lambda: self.engine_.C.double().cpu().numpy()
        while True:
            if eng.oom_guard:
                bad = eng.failed_step(final=eng.n_iter >= cfg.max_iter)
                if bad is not None:
                    c_host, c0 = eng.rollback(bad), eng.c0
                    n_back = eng.n_iter
                    chunk = _retry_chunk(eng.chunk_rows, n_local)
                    self._retired.append(weakref.ref(eng))
                    eng = self.engine_ = None
                    _release(dev)
                    if comm.is_root:
                        print(f"[fcm] out of memory in iteration {n_back + 1}; continuing "
                              f"streamed with chunk_rows={chunk}", flush=True)
                    eng, _ = self._build_engine(x_local, dev, comm, n_global, row_offset, n_local,
                                                c_host, n_back, m, chunk)
                    eng.c0 = c0
                    self.engine_ = eng
                    continue
            if eng.n_iter >= cfg.max_iter:
                break
            if eng.oom_guard:
                eng.save_state()
            eng.step()
            if eng.oom_guard:
                eng.post_flag()
            n_iter = eng.n_iter
            if eng.shift is not None:
                if eng.oom_guard and eng.failed_step(final=True) is not None:
                    continue
                sv = float(eng.shift.item())
                history.append({"iter": n_iter, "shift": sv})
                if sv <= cfg.tol:
                    break
            if ckpt.due(n_iter):
                if eng.oom_guard and eng.failed_step(final=True) is not None:
                    continue
                ckpt.maybe_save(n_iter, centers_host)
            faults.maybe_fail(str(n_iter), comm.rank, kinds=("crash",))
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
            n_global=n_global, streamed=eng.streamed)
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
                           self.cfg.fcm_nan_to_zero, self.cfg.backend, self.cfg.fcm_distances)
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
