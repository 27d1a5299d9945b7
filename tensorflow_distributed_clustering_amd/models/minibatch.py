"""Distributed mini-batch K-Means (Sculley 2010; sklearn ``MiniBatchKMeans`` semantics).

BASELINE config 4 ("Mini-batch K-Means N=1B D=64 K=4096, streamed shards sized for 288 GB
HBM per GPU").  The reference has no mini-batch algorithm; its only answer to large N was
to cluster independent batches and *average* their centers without aligning them
(`scripts/distribuitedClustering.py:296-318`), which is statistically wrong.

Per step every rank takes ``batch_size`` rows of its shard (uniform random rows of a
resident shard, or the next chunk of a streamed/generated shard), runs the same HIP
assign + update kernels as Lloyd on the batch, and ONE packed all-reduce combines the
batch sums/counts.  Each center then moves by the per-center learning rate 1/v_k:

    c_k <- (v_k c_k + S_k) / (v_k + n_k),   v_k <- v_k + n_k

(v_k = points ever assigned to k), i.e. every center is the running mean of the points it
has absorbed -- identical on all ranks, no broadcast needed.
"""
from __future__ import annotations

import time
from typing import Optional

import torch

from ..config import ClusterConfig
from ..data.stream import ResidentSource
from ..ops import acc_dtype_for, make_lloyd_ops
from ..parallel.dist import Comm, local_comm
from ..utils import faults
from ..utils.checkpoint import RunCheckpointer
from ..utils.timers import DeviceTimer, sync
from .init import init_centers, init_centers_from_source
from .kmeans import ClusterResult, _shard_geometry


class MiniBatchStepper:
    """Resident state of a distributed mini-batch run; ``step()`` is one mini-batch update
    (sample/stream a batch, HIP assign+update on it, one all-reduce, Sculley update)."""

    def __init__(self, source, cfg: ClusterConfig, comm: Comm, n_global: int, row_offset: int,
                 init_centers_=None):
        if cfg.batch_size <= 0:
            cfg = cfg.replace(batch_size=1 << 16)
        self.cfg, self.comm = cfg, comm
        self.n_global, self.row_offset = n_global, row_offset
        k = self.k = cfg.n_clusters
        if isinstance(source, torch.Tensor):
            dev = source.device
            self.local = make_lloyd_ops(source, k, cfg.dtype, cfg.backend, cfg.empty_cluster,
                                        cfg.deterministic)
            self.source = ResidentSource(self.local.x, self.local.layout, row_offset)
            self.d = int(source.shape[1])
            self.c0 = init_centers(cfg.init, source, row_offset, n_global, k, comm, cfg.seed,
                                   given=init_centers_, kpp_max_k=cfg.kpp_max_k,
                                   kpp_sample_per_k=cfg.kpp_sample_per_k,
                                   kpp_sample_min=cfg.kpp_sample_min)
        else:
            dev = torch.device(getattr(source, "device", "cpu"))
            self.source = source
            self.d = int(source.d)
            self.local = make_lloyd_ops(torch.zeros(1, self.d, device=dev), k, cfg.dtype,
                                        cfg.backend, cfg.empty_cluster, cfg.deterministic)
            self.c0 = init_centers_from_source(cfg.init, source, row_offset, n_global, k, comm,
                                               cfg.seed, given=init_centers_, d=self.d,
                                               kpp_max_k=cfg.kpp_max_k,
                                               kpp_sample_per_k=cfg.kpp_sample_per_k,
                                               kpp_sample_min=cfg.kpp_sample_min)
        self.device = dev
        self.n_local = int(self.source.n_rows)
        d = self.d
        self.C = self.c0.to(self.local.c_dtype).clone().contiguous()
        self.local.prepare(self.C)
        acc = acc_dtype_for(cfg.dtype, k, d)
        self.buf = torch.zeros(k * d + k, dtype=acc, device=dev)
        self.sums, self.counts = self.buf[: k * d].view(k, d), self.buf[k * d:]
        self.v = torch.zeros(k, dtype=torch.float64, device=dev)
        self.batch_rows = B = min(cfg.batch_size, self.n_local)
        self.blabels = torch.zeros(B, dtype=torch.int32, device=dev)
        self.gen = torch.Generator(device=dev).manual_seed(cfg.seed * 1000003 + comm.rank)
        self._stream_iter = None
        self.shift = None
        self._shift_buf = None
        self.n_iter = 0

    def snapshot(self) -> dict:
        """Restart state (bench.py: timed steps from the init): centres and per-centre counts."""
        return {"C": self.C.clone(), "v": self.v.clone(), "n_iter": self.n_iter}

    def rewind(self, snap: dict):
        self.C.copy_(snap["C"])
        self.v.copy_(snap["v"])
        self.local.prepare(self.C)
        self.n_iter = snap["n_iter"]

    @property
    def resident(self) -> bool:
        return isinstance(self.source, ResidentSource)

    def next_batch(self) -> torch.Tensor:
        if self.resident:
            idx = torch.randint(self.n_local, (self.batch_rows,), generator=self.gen,
                                device=self.device)
            return self.source.rows(idx)
        for _ in range(2):
            if self._stream_iter is None:
                self._stream_iter = self.source.chunks(self.batch_rows)
            try:
                return next(self._stream_iter)[1]
            except StopIteration:
                self._stream_iter = None  # next epoch over the shard
        raise RuntimeError("empty source")

    def _indexed(self) -> bool:
        """Resident shard on the bf16 MFMA path: sample row *indices* and let the kernels
        read the rows in place (no [B, D] gather copy per step)."""
        sup = getattr(self.local, "supports_indexed", None)
        return self.resident and self.device.type == "cuda" and sup is not None and sup()

    def step(self):
        if self._indexed():
            idx = torch.randint(self.n_local, (self.batch_rows,), generator=self.gen,
                                device=self.device, dtype=torch.int32)
            # the all-reduce buffer is cleared by the update's first kernel (no fill launch)
            self.local.step_indexed(self.C, idx, self.blabels, None, self.sums, self.counts,
                                    zero_first=self.buf)
        else:
            self.buf.zero_()
            batch = self.next_batch()
            self.local.bind(batch).step(self.C, self.blabels[: batch.shape[0]], None, self.sums,
                                        self.counts)
        self._apply()

    def step_on(self, batch: torch.Tensor):
        """One mini-batch update on rows the caller supplies (``partial_fit``; online /
        streaming clustering).  Collective: every rank calls it with its own batch."""
        dt, width = self.local.layout
        if not (batch.dtype == dt and batch.shape[1] == width and batch.is_contiguous()):
            xb = torch.zeros(batch.shape[0], width, dtype=dt, device=self.device)
            xb[:, : min(width, batch.shape[1])] = batch[:, :width]
            batch = xb
        if self.blabels.numel() < batch.shape[0]:
            self.blabels = torch.zeros(batch.shape[0], dtype=torch.int32, device=self.device)
        self.buf.zero_()
        self.local.bind(batch).step(self.C, self.blabels[: batch.shape[0]], None, self.sums,
                                    self.counts)
        self._apply()

    def _apply(self):
        """All-reduce the batch partials and move the centres (Sculley)."""
        self.comm.allreduce_bucketed_(self.buf, 64 << 20)
        if hasattr(self.local, "sculley"):
            if self._shift_buf is None:
                self._shift_buf = torch.zeros(1, dtype=torch.float32, device=self.device)
            self._shift_buf.zero_()
            self.local.sculley(self.sums, self.counts, self.C, self.v, self._shift_buf)
            self.shift = self._shift_buf
            self.n_iter += 1
            return
        C64 = self.C.double()
        cnt = self.counts.double()
        nv = self.v + cnt
        upd = (cnt > 0)[:, None]
        newc = (self.v[:, None] * C64 + self.sums.double()) / nv.clamp_min(1.0)[:, None]
        self.shift = ((newc - C64) ** 2).sum(1).masked_fill(~upd[:, 0], 0).max()
        self.C.copy_(torch.where(upd, newc, C64).to(self.C.dtype))
        self.v = nv
        self.local.prepare(self.C)
        self.n_iter += 1

    def label_pass(self):
        dev = self.device
        labels = torch.zeros(self.n_local, dtype=torch.int32, device=dev)
        mind = torch.zeros(self.n_local, dtype=torch.float64 if self.local.c_dtype == torch.float64
                           else torch.float32, device=dev)
        for start, chunk in self.source.chunks(max(self.batch_rows, 1 << 20)):
            s = start - self.source.row_offset
            e = s + chunk.shape[0]
            self.local.bind(chunk).assign(self.C, labels[s:e], mind[s:e])
        self.local.unbind()
        return labels, self.comm.sum_scalar(float(mind.double().sum()))


class MiniBatchKMeans:
    def __init__(self, cfg: ClusterConfig, comm: Optional[Comm] = None, device=None):
        if cfg.batch_size <= 0:
            cfg = cfg.replace(batch_size=1 << 16)
        self.cfg = cfg
        self.comm = comm
        self.device = device
        self.result_: Optional[ClusterResult] = None

    @property
    def cluster_centers_(self):
        if self.result_ is None and getattr(self, "engine_", None) is not None:
            return self.engine_.C.double().cpu().numpy()  # partial_fit state
        return self.result_.centers

    def partial_fit(self, x_batch, init_centers_=None) -> "MiniBatchKMeans":
        """Online update from one batch of rows (sklearn ``partial_fit``): the first call
        initialises the centres from that batch (``cfg.init``; it needs >= K rows), every
        call then applies one Sculley update with the batch.  Multi-rank: every rank calls
        it with its own batch (one all-reduce per call)."""
        cfg = self.cfg
        x = torch.as_tensor(x_batch)
        dev = torch.device(self.device) if self.device is not None else (
            self.comm.device if self.comm is not None else x.device)
        x = x.to(dev)
        if self.comm is None:
            self.comm = local_comm(dev)
        eng = getattr(self, "engine_", None)
        if eng is None:
            n_global, row_offset = _shard_geometry(int(x.shape[0]), self.comm)
            eng = self.engine_ = MiniBatchStepper(x, cfg.replace(batch_size=int(x.shape[0])),
                                                  self.comm, n_global, row_offset,
                                                  init_centers_)
        eng.step_on(x)
        self.result_ = None  # centres moved: cluster_centers_ reads the live state
        return self

    def predict(self, x):
        """Labels of new rows against the current centres."""
        from ..serving import ClusterPredictor
        x = torch.as_tensor(x)
        return ClusterPredictor(self.cluster_centers_, self.cfg.dtype, x.device,
                                self.cfg.backend).predict(x)

    def fit(self, x_local, init_centers_=None, n_global=None, row_offset=None) -> "MiniBatchKMeans":
        cfg = self.cfg
        if cfg.spherical:
            raise ValueError("spherical=True is implemented for KMeans (Lloyd) only")
        t0 = time.perf_counter()
        if hasattr(x_local, "chunks"):
            dev = torch.device(getattr(x_local, "device", "cpu"))
        else:
            x_local = torch.as_tensor(x_local)
            dev = torch.device(self.device) if self.device is not None else (
                self.comm.device if self.comm is not None else x_local.device)
            x_local = x_local.to(dev)
        if self.comm is None:
            self.comm = local_comm(dev)
        comm = self.comm
        n_local = int(x_local.n_rows if hasattr(x_local, "n_rows") else x_local.shape[0])
        if n_global is None or row_offset is None:
            n_global, row_offset = _shard_geometry(n_local, comm)
        sync(dev)
        initialization_time = time.perf_counter() - t0

        t1 = time.perf_counter()
        ckpt = RunCheckpointer(cfg, comm, "miniBatchKMeans")
        d = int(x_local.d if hasattr(x_local, "d") else x_local.shape[1])
        resumed = ckpt.load_for_resume(cfg.n_clusters, d)
        if resumed is not None:
            init_centers_ = resumed.centers
        eng = MiniBatchStepper(x_local, cfg, comm, n_global, row_offset, init_centers_)
        if resumed is not None:
            # per-center counts come back exactly; the batch sampler is re-seeded from the
            # iteration count (statistically equivalent, not the uninterrupted stream)
            eng.n_iter = resumed.n_iter
            if "counts" in resumed.arrays:
                eng.v = torch.as_tensor(resumed.arrays["counts"], dtype=torch.float64, device=dev)
            eng.gen.manual_seed(cfg.seed * 1000003 + comm.rank + 7919 * resumed.n_iter)
        sync(dev)
        setup_time = time.perf_counter() - t1

        timer = DeviceTimer(dev)
        timer.start()
        history = []
        centers_host = lambda: eng.C.double().cpu().numpy()
        counts_host = lambda: {"counts": eng.v.cpu().numpy()}
        for _ in range(max(0, cfg.max_iter - eng.n_iter)):
            eng.step()
            n = eng.n_iter
            if cfg.tol > 0 or (cfg.log_every and n % cfg.log_every == 0):
                sv = float(eng.shift)
                history.append({"iter": n, "shift": sv})
                if cfg.tol > 0 and sv <= cfg.tol:
                    break
            ckpt.maybe_save(n, centers_host, counts_host)
            faults.maybe_fail(str(n), comm.rank)
        computation_time = timer.stop()
        ckpt.maybe_save(eng.n_iter, centers_host, counts_host, final=True)

        labels, inertia = eng.label_pass() if cfg.label_pass else (None, None)
        self.engine_ = eng
        self.result_ = ClusterResult(
            centers=eng.C.double().cpu().numpy(), init_centers=eng.c0.cpu().numpy(),
            labels=labels, counts=eng.v.cpu().numpy(), n_iter=eng.n_iter, inertia=inertia,
            setup_time=setup_time, initialization_time=initialization_time,
            computation_time=computation_time, backend=eng.local.name, history=history,
            n_global=n_global, streamed=not eng.resident)
        self.points_processed_ = eng.n_iter * eng.batch_rows * comm.world_size
        return self
