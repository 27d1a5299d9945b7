"""Distributed Lloyd K-Means (data-parallel over points, replicated centroids).

Reference: ``distribuited_k_means`` (`scripts/distribuitedClustering.py:180-294`).
Per iteration the reference ran one TF session step that (1) materialised [N_g,K,D]
tiles per GPU, (2) gathered per-cluster means with K dynamic-shape Where/Gather chains,
(3) copied labels to the host for a CPU bincount, (4) reduced everything on a CPU
parameter server, and then (5) re-ran the whole distance computation for an untimed
CPU label pass (`:277-282`).  When the data did not fit, it split N into batches that
were clustered *independently* and averaged their centers (`:296-360`).

Here one iteration on each rank is:

    comm_buf.zero_()                               # [sums K*D | counts K], one flat buffer
    for chunk in source.chunks(chunk_rows):        # one chunk when the shard is resident
        local.bind(chunk).step(C, labels, ..., sums, counts)   # N1 assign + N2 update (HIP)
    all_reduce(comm_buf)                           # ONE RCCL call over xGMI (gloo on CPU)
    local.finalize(sums, counts, C)                # N3 divide + next-iteration operand prep

so a streamed pass (host-resident or generated data, larger than HBM) is the *exact*
Lloyd step -- partial sums accumulate over all chunks before the single all-reduce.
Labels come out of the same kernel that feeds the update; a final label pass against
the *final* centroids (what the reference returns as ``cluster_idx``) runs untimed.
"""
from __future__ import annotations

import gc
import math
import time
import weakref
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import torch

from ..config import ClusterConfig
from ..data.stream import HostSource, ResidentSource, plan_chunk_rows, plan_resident_rows
from ..ops import (NativeUpdate, acc_dtype_for, lloyd_fixed_extra, lloyd_layout, lloyd_row_extra,
                   make_lloyd_ops)
from ..parallel.dist import Comm, join_counts, local_comm
from ..utils import faults
from ..utils.checkpoint import RunCheckpointer
from ..utils.timers import DeviceTimer, sync
from .init import floyd_sample, init_centers, init_centers_from_source


@dataclass
class ClusterResult:
    centers: np.ndarray                 # [K, D] float64 (host)
    init_centers: np.ndarray            # [K, D] float64
    labels: Optional[torch.Tensor]      # this rank's labels (int32, on device)
    counts: Optional[np.ndarray]        # [K] global cluster sizes of the last update
    n_iter: int
    inertia: Optional[float]
    setup_time: float
    initialization_time: float
    computation_time: float
    backend: str = ""
    history: List[dict] = field(default_factory=list)
    n_global: int = 0
    streamed: bool = False

    @property
    def points_per_sec(self) -> float:
        return self.n_global * self.n_iter / self.computation_time if self.computation_time > 0 else 0.0

    @property
    def iters_per_sec(self) -> float:
        return self.n_iter / self.computation_time if self.computation_time > 0 else 0.0


def _release(dev: torch.device):
    """Return the memory of dropped engines / sources to the device before a retry
    (reference cycles through exception frames are collected first)."""
    gc.collect()
    if dev.type == "cuda":
        torch.cuda.empty_cache()


def _retry_chunk(chunk: int, n_local: int) -> int:
    """Streamed chunk rows after an OOM: half the previous chunk; from a resident shard,
    a quarter of it (the stream holds two device slots, so they take half the shard)."""
    return max(1024, (chunk or n_local // 2) // 2)


def _shard_geometry(n_local: int, comm: Comm):
    sizes = comm.all_gather_sizes(int(n_local))
    return int(sum(sizes)), int(sum(sizes[: comm.rank]))


class OomGuard:
    """Mid-run OOM rollback state shared by the Lloyd and FCM engines.

    A rank that runs out of memory in its local step sets the flag slot of the packed
    all-reduce buffer, so every rank learns it from the same collective.  The flag of each
    step is copied to pinned host memory asynchronously; :meth:`failed_step` reads the flags
    in order, at most ``OOM_LAG`` steps behind the host (the host never waits for the step
    it just queued, so launches stay ahead of the GPU), or all of them with ``final``.  The
    pre-step centroids of the last ``OOM_LAG + 2`` steps are kept, so a flag seen late
    still rolls back to the state before the failed step.  Engines provide ``rsag``, ``C``
    (+ ``C_pad``/``_r0``/``_kr`` under rsag), ``buf``, ``oom_flag``, ``device``, ``n_iter``
    and ``centers()``."""

    OOM_LAG = 3

    def _oom_alloc(self):
        """Ring of pre-step centroids, pinned flag slots and events (allocated at setup,
        never inside the timed loop: a pinned allocation costs ~1 ms)."""
        src = self.C_pad[self._r0: self._r0 + self._kr] if self.rsag else self.C
        R = self.OOM_LAG + 2
        self._ring = [torch.empty_like(src) for _ in range(R)]
        self._ring_iter = [-1] * R
        self._flag_host = torch.zeros(R, dtype=self.buf.dtype,
                                      pin_memory=self.device.type == "cuda")
        self._flag_ev = ([torch.cuda.Event() for _ in range(R)]
                         if self.device.type == "cuda" else [None] * R)
        self._flag_step = [-1] * R
        self._checked = -1  # every step <= this one is known to have completed cleanly

    def save_state(self):
        """Keep the pre-step centroids (this rank's slice under rsag) for a rollback."""
        if getattr(self, "_ring", None) is None:
            self._oom_alloc()
        src = self.C_pad[self._r0: self._r0 + self._kr] if self.rsag else self.C
        slot = self.n_iter % len(self._ring)
        self._ring[slot].copy_(src)
        self._ring_iter[slot] = self.n_iter

    def post_flag(self):
        """After step(): queue the copy of this step's OOM flag (no host sync)."""
        step = self.n_iter - 1
        slot = step % len(self._ring)
        if self.device.type == "cuda":
            self._flag_host[slot:slot + 1].copy_(self.oom_flag, non_blocking=True)
            self._flag_ev[slot].record()
        else:
            self._flag_host[slot:slot + 1].copy_(self.oom_flag)
        self._flag_step[slot] = step

    def failed_step(self, final: bool = False) -> Optional[int]:
        """Index (0-based) of the first step whose flag is set, among the steps not yet
        checked that are ``OOM_LAG`` or more steps old (``final``: all of them -- a host
        sync on the last step)."""
        if getattr(self, "_ring", None) is None:
            return None
        R = len(self._ring)
        upto = self.n_iter - 1 if final else self.n_iter - 1 - self.OOM_LAG
        while self._checked < upto:
            n = self._checked + 1
            slot = n % R
            if self._flag_step[slot] == n:
                ev = self._flag_ev[slot]
                if ev is not None:
                    ev.synchronize()
                if float(self._flag_host[slot]) > 0:
                    return n
            self._checked = n
        return None

    # ------------------------------------------------------------ untimed warm-up step
    _warming = False
    warmup_ok = True  # engines with incremental state a discarded step would corrupt: off

    def warmup(self, force: bool = False):
        """One step whose result is discarded (the centroids and the iteration count are
        restored): the first launch of each step kernel loads its code object and sizes
        its grid (~2.5 ms at the reference's N=25M, K=3 -- more than ten iterations), a
        setup cost that belongs in setup_time, not in the timed iterations.  Resident,
        replicated-centroid engines on a GPU only (a streamed pass would cost a full
        transfer; rsag state is sliced across ranks)."""
        skip = (not self.warmup_ok or self.streamed or getattr(self, "rsag", False)
                or getattr(self, "_graph", None) is not None
                or (self.device.type != "cuda" and not force))
        if self.comm.collective:
            # the step is collective: warm up only if every rank can (a rank whose planner
            # chose streaming would otherwise leave the others waiting in the all-reduce)
            skip = self.comm.max_scalar(1.0 if skip else 0.0) > 0.0
        if skip:
            return
        c0, n0 = self.C.clone(), self.n_iter
        self._warming = True
        try:
            self.step()
        finally:
            self._warming = False
        self.C.copy_(c0)
        self.local.prepare(self.C)
        self.n_iter = n0
        # the delta update's running totals now describe the discarded step's assignment:
        # timed iteration 1 must re-sum every row, as the reference's first iteration does
        # (`scripts/distribuitedClustering.py:277-280`), not take a delta over a warm-up
        if getattr(self, "delta", None) is not None:
            self.delta.reset()

    def rollback(self, step: int) -> np.ndarray:
        """Centroids at the start of ``step`` (replicated, host fp64); resets n_iter."""
        slot = step % len(self._ring)
        assert self._ring_iter[slot] == step, "rollback state of the failed step is gone"
        prev = self._ring[slot]
        if self.rsag:
            self.C_pad[self._r0: self._r0 + self._kr].copy_(prev)
            self._c_synced = False
        else:
            self.C.copy_(prev)
        self.n_iter = step
        self._checked = step - 1
        return self.centers().double().cpu().numpy()


class LloydEngine(OomGuard):
    """Resident state of one distributed Lloyd run: operands, centroids, buffers.

    ``source`` is a device tensor (the resident shard) or a chunk source from
    :mod:`..data.stream`.  ``step()`` is exactly one iteration (assign + update +
    all-reduce + finalize); it is what ``bench.py`` times and what :meth:`KMeans.fit`
    loops over.
    """

    def __init__(self, source, cfg: ClusterConfig, comm: Comm, n_global: int, row_offset: int,
                 init_centers_=None, chunk_rows: int = 0, defer_init: bool = False):
        self.cfg, self.comm = cfg, comm
        self.n_global, self.row_offset = n_global, row_offset
        k = cfg.n_clusters
        self.k = k
        if isinstance(source, torch.Tensor):
            if cfg.spherical:
                # cosine K-Means: on unit vectors ||x - c||^2 = 2 - 2 cos(x, c) for unit c,
                # so the L2 kernels rank by cosine once rows and centroids are normalised
                n = source.float().norm(dim=1, keepdim=True).clamp_min_(1e-30)
                source = (source.float() / n).to(source.dtype)
            x0 = source
            self.local = make_lloyd_ops(source, k, cfg.dtype, cfg.backend, cfg.empty_cluster,
                                        cfg.deterministic, cfg.kgroup_bytes, cfg.fp8_recheck,
                                        cfg.exact_assign)
            self.source = ResidentSource(self.local.x, self.local.layout, row_offset)
            self.local.x = self.source.x
            self.device = source.device
            self.d = int(source.shape[1])
            self.n_local = int(source.shape[0])
        else:
            if cfg.spherical:
                raise ValueError("spherical K-Means needs a resident shard (normalised once)")
            self.source = source
            self.device = torch.device(getattr(source, "device", comm.device))
            self.d = int(source.d)
            self.n_local = int(source.n_rows)
            probe = torch.zeros(1, self.d, dtype=torch.float32, device=self.device)
            self.local = make_lloyd_ops(probe, k, cfg.dtype, cfg.backend, cfg.empty_cluster,
                                        cfg.deterministic, cfg.kgroup_bytes, cfg.fp8_recheck,
                                        cfg.exact_assign)
            if tuple(self.local.layout) != tuple(source.layout):
                raise ValueError(f"source layout {source.layout} != kernel layout {self.local.layout}")
            x0 = None
        self.chunk_rows = chunk_rows
        self.streamed = not isinstance(self.source, ResidentSource) or chunk_rows > 0
        dev = self.device
        self._x0 = x0
        self._init_given = init_centers_
        acc = acc_dtype_for(cfg.dtype, k, self.d)
        # deterministic native update: int64 fixed-point partials (ops.NativeUpdate), the
        # scale agreed on by the ranks in init_centroids
        self.fixed = bool(self.local.fixed_point()) and self.fixed_ok
        if self.fixed:
            acc = torch.int64
        # fp32 partial sums: the counts also travel as exact integer halves (hi, lo) in the
        # same buffer (parallel/dist.split_counts); without the kernel support: fp64 buffer
        self.count_split = (acc == torch.float32 and self.exact_counts_ok
                            and self.local.supports_count_split())
        if acc == torch.float32 and not self.count_split:
            acc = torch.float64
        self.rsag = (not self.fixed) and self._use_rsag(
            comm, cfg, k * self.d * torch.tensor([], dtype=acc).element_size())
        W = comm.world_size
        if self.rsag:
            align = math.lcm(max(1, self.local.row_align), W)
            kpad = -(-k // align) * align
            self.local.pad_rows(kpad)
        else:
            kpad = k
        self.kpad = kpad
        # delta update: only the rows whose label changed move between fp64 running totals.
        # Under rsag each rank keeps the totals of its own slice of centroid rows (the
        # reduce-scatter hands it exactly those deltas); the moved count and the signed
        # count deltas ride in the all-reduced tail, so every rank picks the same mode
        self.delta = None
        if (cfg.update != "full" and self.delta_ok and not self.streamed
                and cfg.empty_cluster in ("keep", "nan", "zero")):
            g_rows = None
            if self.rsag:
                r0 = comm.rank * (kpad // W)
                g_rows = max(0, min(k, r0 + kpad // W) - r0)
            self.delta = self.local.make_delta(self.n_local, k, self.d, cfg.delta_refresh,
                                               cfg.delta_theta, cfg.empty_cluster, g_rows)
        # 'nan_any' (script compat): K extra "empty on this rank" flags ride in the same
        # all-reduce; a cluster empty on ANY rank becomes NaN everywhere, like the
        # reference's per-GPU reduce_mean of an empty gather (`distribuitedClustering.py:240,248`)
        self.nan_any = cfg.empty_cluster == "nan_any"
        # buf = [sums kpad*D | counts kpad | (hi kpad | lo kpad) | (flags kpad)]: the sums
        # block is what a reduce-scatter splits by rank; the small tail is all-reduced
        nsmall = 1 + (2 if self.count_split else 0) + (1 if self.nan_any else 0)
        # + 1 slot: rows whose label changed this step (delta update: picks the next mode;
        #   always there, so every rank's buffer has the same layout before the ranks agree
        #   on the update mode in init_centroids)
        # + 1 slot: "a rank ran out of memory in this step's local work" (oom_pending)
        self.oom_guard = bool(cfg.oom_recovery) and self.oom_guard_ok
        ntail = 1 + (1 if self.oom_guard else 0)
        self.buf = torch.zeros(kpad * self.d + nsmall * kpad + ntail, dtype=acc, device=dev)
        self.sums_pad = self.buf[: kpad * self.d].view(kpad, self.d)
        self.sums = self.sums_pad[:k]
        self.small = self.buf[kpad * self.d:]
        self.counts = self.small[:k]
        row = 1
        self.cnt_hi = self.cnt_lo = None
        if self.count_split:
            self.cnt_hi = self.small[kpad: kpad + k]
            self.cnt_lo = self.small[2 * kpad: 2 * kpad + k]
            self.local.set_count_split(self.cnt_hi, self.cnt_lo)
            row = 3
        self.empty_flags = self.small[row * kpad: row * kpad + k] if self.nan_any else None
        self.oom_flag = self.buf[-1:] if self.oom_guard else None
        off = kpad * self.d + nsmall * kpad
        self.moved_slot = self.buf[off: off + 1]
        self.C_pad = torch.zeros(kpad, self.d, dtype=self.local.c_dtype, device=dev)
        self.C = self.C_pad[:k]
        if self.rsag:
            kr = kpad // W
            self._kr = kr
            self._r0 = comm.rank * kr
            self._rs_out = torch.zeros(kr, self.d, dtype=acc, device=dev)
            ops_ = self.local.gather_operands()
            self._gathered = ops_ if ops_ is not None else [self.C_pad]
            self._c_synced = True
        self.labels = torch.zeros(self.n_local, dtype=torch.int32, device=dev)
        if hasattr(self.local, "skip_step_labels"):
            # the fit's final label pass writes the labels: the steps need only the sums
            self.local.skip_step_labels = bool(cfg.label_pass)
        mdt = torch.float64 if self.local.c_dtype == torch.float64 else torch.float32
        self.mind = torch.zeros(self.n_local, dtype=mdt, device=dev) if cfg.compute_inertia else None
        self.need_shift = cfg.tol > 0 or cfg.log_every > 0
        self.shift = torch.zeros(1, dtype=torch.float32, device=dev) if self.need_shift else None
        self.bucket_bytes = cfg.bucket_kb << 10
        # resident sorted update: the step's zero fill of buf rides in the update's first
        # kernel (one launch less per step; the small-shard step is launch-bound)
        upd = getattr(self.local, "update", None)
        self._zero_fused_full = (isinstance(upd, NativeUpdate) and upd.fuses_zero()
                                 and not self.streamed and type(self) is LloydEngine)
        if self._zero_fused_full:
            upd.zero_buf = self.buf
        self._set_delta(self.delta)
        self.n_iter = 0
        self.c0 = None
        if self.oom_guard:
            self._oom_alloc()
        if not defer_init:
            self.init_centroids()

    # delta centroid update allowed (subclasses with their own step: off)
    delta_ok = True
    # fixed-point (int64) buffers for the deterministic update (subclasses that do float
    # arithmetic on buf: off)
    fixed_ok = True
    # exact count halves in the buffer (subclasses with their own count bookkeeping: off)
    exact_counts_ok = True
    # mid-run OOM flag in the buffer (subclasses with their own step: off)
    oom_guard_ok = True
    # reduce-scatter / all-gather mode allowed (subclasses that read the whole buf: off)
    rsag_ok = True
    RSAG_MIN_BYTES = 32 << 20

    def _use_rsag(self, comm: Comm, cfg: ClusterConfig, sums_bytes: int) -> bool:
        if not comm.collective or not self.rsag_ok:
            return False
        if cfg.comm_mode == "rsag":
            return True
        return cfg.comm_mode == "auto" and sums_bytes >= self.RSAG_MIN_BYTES

    def exact_counts(self) -> torch.Tensor:
        """Global cluster sizes of the last update (fp64, exact past 2^24)."""
        if self.delta is not None and self.rsag:
            # each rank holds the totals of its slice: gather them (collective)
            part = torch.zeros(self._kr, dtype=torch.float64, device=self.device)
            part[: self.delta.gk] = self.delta.counts
            full = torch.zeros(self.kpad, dtype=torch.float64, device=self.device)
            self.comm.all_gather_(full, part)
            return full[: self.k].clone()
        if self.delta is not None:
            return self.delta.counts.clone()
        if self.count_split:
            return join_counts(self.cnt_hi, self.cnt_lo)
        return self.counts.double()

    def centers(self) -> torch.Tensor:
        """The full centroid table (rsag ranks only finalise their slice: gather the rest)."""
        if self.rsag and not self._c_synced:
            part = self.C_pad[self._r0: self._r0 + self._kr].contiguous()
            self.comm.all_gather_(self.C_pad, part)
            self._c_synced = True
        return self.C

    def _set_delta(self, delta):
        self.delta = delta
        # the native diff kernel clears buf (the full sorted update's hist kernel otherwise)
        self._zero_fused = (bool(getattr(delta, "native", False)) if delta is not None
                            else self._zero_fused_full)

    def _agree_update_mode(self):
        """Every rank runs the same update mode (the totals are replicated, or sliced by
        rank under rsag): the delta update only if every rank supports it (a rank whose
        planner streams its shard cannot).  Collective."""
        ok = self.delta is not None
        if self.comm.collective:
            ok = self.comm.max_scalar(0.0 if ok else 1.0) == 0.0
        if not ok:
            self._set_delta(None)
        if self.cfg.update == "delta" and self.delta is None:
            raise ValueError("update='delta' needs a resident shard on every rank, a sorted/LDS "
                             "native update or the torch ops, K <= 65536, empty_cluster in "
                             "keep/nan/zero and no bounded mode")

    def _agree_fixed_scale(self):
        """Deterministic update: the fixed-point scale 2^S of the int64 partials, from the
        global max |x| and N (collective; one max-reduction, plus one pass over a streamed
        shard).  Every rank uses the same S, so the int64 all-reduce adds like terms."""
        from ..ops import fixed_point_scale
        if isinstance(self.source, ResidentSource):
            xs = [self.local.x]
        else:
            xs = (chunk for _, chunk in self._chunks())
        m = 0.0
        wide = False
        for xc in xs:
            wide = wide or xc.dtype == torch.float64
            if xc.numel():
                # a NaN / inf row propagates as inf: fixed_point_scale names it
                v = xc[:, : self.d].abs().max()
                m = max(m, float(v) if bool(torch.isfinite(v)) else math.inf)
        m = self.comm.max_scalar(m)
        scale = fixed_point_scale(m, self.n_global, elem32=not wide)
        self.local.set_fixed_scale(scale)
        if self.delta is not None:
            self.delta.fixed_scale = scale
        self.fixed_scale = scale

    def init_centroids(self):
        """Centroid init (collective: every rank calls it, in the same order).  Kept out
        of the constructor's local allocations so a setup OOM can be agreed on first."""
        cfg, comm, k = self.cfg, self.comm, self.k
        self._agree_update_mode()
        if self.fixed:
            self._agree_fixed_scale()
        if self._x0 is not None:
            c0 = init_centers(cfg.init, self._x0, self.row_offset, self.n_global, k, comm,
                              cfg.seed, given=self._init_given, kpp_max_k=cfg.kpp_max_k,
                              kpp_sample_per_k=cfg.kpp_sample_per_k,
                              kpp_sample_min=cfg.kpp_sample_min)
        else:
            c0 = init_centers_from_source(cfg.init, self.source, self.row_offset, self.n_global,
                                          k, comm, cfg.seed, given=self._init_given, d=self.d,
                                          kpp_max_k=cfg.kpp_max_k,
                                          kpp_sample_per_k=cfg.kpp_sample_per_k,
                                          kpp_sample_min=cfg.kpp_sample_min)
        if cfg.spherical:
            c0 = c0 / c0.norm(dim=1, keepdim=True).clamp_min(1e-30)
        self.c0 = c0
        self.C.copy_(c0.to(self.local.c_dtype))  # never alias c0
        self.local.prepare(self.C)
        if self.delta is not None:
            self.delta.reset()
        self._x0 = None
        return self

    def _chunks(self):
        return self.source.chunks(self.chunk_rows)

    def step(self, with_inertia: bool = False) -> Optional[float]:
        """One Lloyd iteration.  ``with_inertia``: also return the global inertia of this
        iteration's assignment (the fused distance epilogue writes min distances; costs one
        scalar all-reduce + host sync, so it is only requested at log points)."""
        g = getattr(self, "_graph", None)
        if g is not None and not with_inertia:
            g.replay()
            self.n_iter += 1
            return None
        return self._eager_step(with_inertia)

    def _eager_step(self, with_inertia: bool = False) -> Optional[float]:
        if not self._zero_fused:
            self.buf.zero_()
        mind = self.mind if (with_inertia and self.mind is not None) else None
        try:
            if self.oom_guard and not self._warming:
                faults.maybe_fail(str(self.n_iter + 1), self.comm.rank, kinds=("oom",))
            self._local_step(mind)
        except Exception as e:  # noqa: BLE001 - filtered right below
            if self.oom_flag is None or not faults.is_oom(e):
                raise
            # every rank still joins this step's collectives; the flag makes them all see it
            self.buf.zero_()
            self.oom_flag.fill_(1.0)
            if mind is not None:
                mind.zero_()
        inertia = self.comm.sum_scalar(float(mind.double().sum())) if mind is not None else None
        if self.nan_any:
            self.empty_flags.copy_((self.counts == 0).to(self.buf.dtype))
        if self.rsag:
            self._reduce_scatter_finalize()
        else:
            self.comm.allreduce_bucketed_(self.buf, self.bucket_bytes)
            if self.nan_any:
                self.counts.masked_fill_(self.empty_flags > 0, 0)
            if self.shift is not None:
                self.shift.zero_()
            self._finalize()
        if self.cfg.spherical:  # project the means back to the sphere
            self.centers()
            self.C.div_(self.C.norm(dim=1, keepdim=True).clamp_min_(1e-30))
            self.local.prepare(self.C)
        if self.cfg.empty_cluster == "reseed":
            self._reseed()
        self.n_iter += 1
        return inertia

    def _split(self):
        return (self.cnt_hi, self.cnt_lo) if self.count_split else None

    def _delta_update(self):
        self.delta.update(self.local.x, self.labels, self.sums, self.counts, self._split(),
                          self.moved_slot, self.buf if self._zero_fused else None)

    def _finalize(self):
        if self.delta is not None:
            cm2, cnorm = self.local.bf16_operands()
            self.delta.finalize(self.sums, self.counts, self._split(), self.moved_slot, self.C,
                                self.local.policy, self.shift, cm2, cnorm, self.n_global)
            self.local.after_finalize(self.C)
        else:
            self.local.finalize(self.sums, self.counts, self.C, self.shift)

    # ------------------------------------------------------------ restart from a state
    def snapshot(self) -> dict:
        """The state the iterations can be restarted from (bench.py: the timed steps are
        iterations 1..K from the centroid init, as the reference's computation_time,
        `scripts/distribuitedClustering.py:277-280`, after untimed warm-up steps)."""
        return {"C": self.C_pad.clone(), "n_iter": self.n_iter}

    def rewind(self, snap: dict):
        """Back to :meth:`snapshot`: centroids (every row, replicated), operands, iteration
        count; the delta update starts over with a full step (its running totals describe
        the warm-up's assignment, not one of these centroids)."""
        self.C_pad.copy_(snap["C"])
        self._c_synced = True
        self.local.prepare(self.C)
        if self.delta is not None:
            self.delta.reset()
        self.n_iter = snap["n_iter"]

    def update_stats(self) -> Optional[dict]:
        """Delta-update bookkeeping so far (host read): moved rows summed over the steps
        that had a previous assignment, those steps, full steps, all steps; None without
        the delta update."""
        return self.delta.stats_host() if self.delta is not None else None

    @property
    def update_mode(self) -> str:
        return "delta" if self.delta is not None else "full"

    def phase_fns(self):
        """(name, fn) of one resident step's phases in order (timing breakdowns): the
        buffer fill, assign, local update, all-reduce, finalize."""
        loc = self.local
        if self.delta is not None:
            assign = lambda: loc.assign(self.C, self.labels, None)
            update = self._delta_update
        elif isinstance(getattr(loc, "update", None), NativeUpdate):
            assign = lambda: loc.assign(self.C, self.labels, None)
            update = lambda: loc.update(loc.x, self.labels, self.sums, self.counts)
        else:
            assign = lambda: loc.step(self.C, self.labels, None, self.sums, self.counts)
            update = lambda: None
        return [("zero", self.buf.zero_), ("assign", assign), ("update", update),
                ("allreduce", lambda: self.comm.allreduce_bucketed_(self.buf, self.bucket_bytes)),
                ("finalize", self._finalize)]

    def _local_step(self, mind):
        if self.delta is not None:
            self.local.assign(self.C, self.labels, mind)
            self._delta_update()
        elif not self.streamed:
            self.local.step(self.C, self.labels, mind, self.sums, self.counts)
        else:
            for start, chunk in self._chunks():
                s = start - self.source.row_offset  # chunk starts are source-global
                e = s + chunk.shape[0]
                self.local.bind(chunk).step(self.C, self.labels[s:e],
                                            None if mind is None else mind[s:e],
                                            self.sums, self.counts)
            self.local.unbind()

    def _reduce_scatter_finalize(self):
        """rsag mode: reduce-scatter the sums (rank r gets centroid rows [r0, r0 + kr)),
        all-reduce the small count tail, finalise + operand-prep the own slice, all-gather
        the assign operands (bf16/fp8 tables: 2-4x fewer bytes than the fp32 centroids;
        an all-reduce moves the fp32 sums twice)."""
        comm, k, kr, r0 = self.comm, self.k, self._kr, self._r0
        comm.reduce_scatter_(self._rs_out.view(-1), self.buf[: self.kpad * self.d])
        comm.allreduce_(self.small)
        if self.nan_any:
            self.counts.masked_fill_(self.empty_flags > 0, 0)
        if self.shift is not None:
            self.shift.zero_()
        r1 = min(k, r0 + kr)
        nv = max(0, r1 - r0)
        if self.delta is not None:
            # the slice's deltas (or, on a full step, its sums) into the slice's fp64 totals;
            # ctrl's next mode comes from the all-reduced moved count, the same on every rank
            cm2, cnorm = self.local.bf16_operands()
            split = ((self.cnt_hi[r0:r0 + nv], self.cnt_lo[r0:r0 + nv]) if self.count_split
                     else None)
            self.delta.finalize(self._rs_out[:nv], self.counts[r0:r0 + nv], split,
                                self.moved_slot, self.C_pad[r0:r0 + nv], self.local.policy,
                                self.shift, None if cm2 is None else cm2[r0:r0 + kr],
                                None if cnorm is None else cnorm[r0:r0 + kr], self.n_global)
            if cm2 is None:
                self.local.prep_rows(self.C_pad[r0:r0 + nv], r0, kr)
        else:
            self.local.finalize_rows(self._rs_out[:nv], self.counts[r0:r0 + nv],
                                     self.C_pad[r0:r0 + nv], self.shift, r0, kr)
        for t in self._gathered:
            part = t[r0:r0 + kr].contiguous()
            comm.all_gather_(t, part)
        self._c_synced = self._gathered[0] is self.C_pad
        if self._c_synced:
            self.local.after_gather(self.C)
        if self.shift is not None:
            comm.allreduce_(self.shift, "max")

    # ------------------------------------------------------------ HIP graph replay
    def graphable(self) -> bool:
        """A step is capturable when it is device-only: resident shard (streamed chunks
        loop over host work), no host-side reseed, a CUDA device.  Collectives are
        captured only on request (RCCL graph capture), so by default world_size == 1."""
        return (self.device.type == "cuda" and not self.streamed
                and self.cfg.empty_cluster != "reseed")

    def capture(self, include_collectives: bool = False):
        """Capture one step into a hipGraph (torch.cuda.CUDAGraph); ``step()`` replays it.

        The step is launch-bound for small N (6-8 kernels + an all-reduce per iteration);
        replay removes the per-launch host cost.  Warm-up runs on a side stream first, as
        graph capture requires."""
        if not self.graphable():
            raise RuntimeError("this engine configuration cannot be captured")
        if self.comm.collective and not include_collectives:
            raise RuntimeError("capture with collectives (world_size > 1 or forced) needs "
                               "include_collectives=True")
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        snapshot = (self.C.clone(), self.n_iter)
        with torch.cuda.stream(s):
            self._eager_step()          # warm-up (allocations, kernel attributes, RCCL comms)
        torch.cuda.current_stream(self.device).wait_stream(s)
        self.C.copy_(snapshot[0])
        self.local.prepare(self.C)
        self.n_iter = snapshot[1]
        if self.delta is not None:
            self.delta.reset()  # the warm-up's assignment is not this state's (as warmup())
        settle = getattr(self.local, "settle", None)
        if settle is not None:
            # host-side choices a replay cannot revisit (the x3 prefilter and its listed
            # launch size) are made from the warm-up step's measured state
            settle()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._eager_step()
        # capture does not execute: restore the iteration count, keep C untouched
        self.n_iter = snapshot[1]
        self._graph = g
        return self

    def _reseed(self):
        empty = torch.nonzero(self.counts == 0).flatten().cpu().tolist()
        if not empty:
            return
        self.centers()
        idx = floyd_sample(self.n_global, len(empty), self.cfg.seed + 7919 * (self.n_iter + 1))
        rows = init_centers_from_source("rows", self.source, self.row_offset, self.n_global,
                                        len(empty), self.comm, 0, rows=idx, d=self.d)
        self.C[torch.as_tensor(empty, device=self.C.device)] = rows.to(self.C.dtype)
        self.local.prepare(self.C)

    def label_pass(self) -> Optional[float]:
        """Assign against the current centroids; returns the global inertia if tracked."""
        if not self.streamed:
            self.local.assign(self.C, self.labels, self.mind)
        else:
            for start, chunk in self._chunks():
                s = start - self.source.row_offset
                e = s + chunk.shape[0]
                self.local.bind(chunk).assign(self.C, self.labels[s:e],
                                              None if self.mind is None else self.mind[s:e])
            self.local.unbind()
        if self.mind is None:
            return None
        return self.comm.sum_scalar(float(self.mind.double().sum()))


def build_engine_collective(tag: str, cfg: ClusterConfig, comm: Comm, dev, n_local: int,
                            start_iter: int, chunk: int, make_source, make_engine):
    """Build an engine with collective OOM handling; returns (engine, seconds spent in
    ``make_source``, i.e. loading / uploading the shard).

    The source (the device upload of a resident shard) is created inside the agreement:
    if any rank runs out of memory while uploading or building, every rank frees what it
    holds and retries with the shard streamed from host memory in halved chunks.  The
    reference doubled its batch count on ResourceExhaustedError
    (`scripts/distribuitedClustering.py:331-360`) but clustered the batches independently;
    here the streamed pass is still the exact step.  ``chunk`` > 0 (a mid-run OOM retry)
    streams from the start."""
    t_src = 0.0
    err = None
    for attempt in range(cfg.max_oom_retries + 1):
        err = None
        eng = source = None
        try:
            faults.maybe_fail("setup", comm.rank)  # an injected OOM of the upload
            t = time.perf_counter()
            source, chunk_rows = make_source(chunk)
            sync(dev)
            t_src += time.perf_counter() - t
            chunk = chunk_rows or chunk
            eng = make_engine(source, chunk_rows)
        except Exception as e:  # noqa: BLE001 - filtered right below
            if not faults.is_oom(e):
                raise
            err = e
        if err is not None:
            # the traceback's frames hold the half-built engine and the device copy
            err.__traceback__ = None
        if comm.max_scalar(1.0 if err is not None else 0.0) == 0.0:
            eng.init_centroids()
            eng.n_iter = start_iter
            return eng, t_src
        del eng, source
        _release(dev)
        chunk = _retry_chunk(chunk, n_local)
        if comm.is_root:
            print(f"[{tag}] out of memory while building the engine "
                  f"({type(err).__name__ if err else 'peer rank'}); retrying streamed with "
                  f"chunk_rows={chunk}", flush=True)
    raise err if err is not None else faults.oom_error("out of memory on a peer rank")


class KMeans:
    """sklearn-like front end over the distributed engine.

    >>> km = KMeans(ClusterConfig(n_clusters=8, dtype="fp32")).fit(x)
    >>> km.result_.centers

    ``x_local`` is this rank's row shard: a device tensor (resident), a CPU tensor or
    numpy array (moved to the device, or streamed from host memory when it does not fit
    the HBM budget or ``cfg.chunk_rows`` is set), or a chunk source from
    :mod:`..data.stream`.
    """

    def __init__(self, cfg: ClusterConfig, comm: Optional[Comm] = None, device=None):
        self.cfg = cfg
        self.comm = comm
        self.device = device
        self.result_: Optional[ClusterResult] = None
        self.local_ = None

    @property
    def cluster_centers_(self) -> np.ndarray:
        return self.result_.centers

    @property
    def labels_(self) -> torch.Tensor:
        return self.result_.labels

    def _target_device(self, x):
        if self.device is not None:
            return torch.device(self.device)
        if self.comm is not None:
            return self.comm.device
        if isinstance(x, torch.Tensor):
            return x.device
        return torch.device(getattr(x, "device", "cpu"))

    def _make_source(self, x_local, dev, row_offset, chunk_override: int = 0):
        """(source, chunk_rows): the resident device shard, or a HostSource when the shard
        stays in host memory (it does not fit the HBM budget, or cfg.chunk_rows / an OOM
        retry asks for streaming).  Every dtype streams: the native RowStreamer converts
        host rows into the kernel layout (bf16 / fp32, or fp64 rows as they are) in a
        pinned ring with H2D on a copy stream; the planner keeps the leading rows that fit
        next to the streaming buffers resident."""
        cfg = self.cfg
        want = chunk_override or cfg.chunk_rows
        if hasattr(x_local, "chunks"):
            return x_local, want or (1 << 22)
        if isinstance(x_local, torch.Tensor) and x_local.device.type != "cpu":
            # device data stays where the caller put it: a retry can only re-chunk it
            return x_local.to(dev), want
        xn = x_local.numpy() if isinstance(x_local, torch.Tensor) else np.asarray(x_local)
        if dev.type == "cuda" and cfg.backend != "torch":
            d = xn.shape[1]
            layout = lloyd_layout(cfg.dtype, d)
            es = torch.tensor([], dtype=layout[0]).element_size()
            row_bytes = layout[1] * es
            # per-row / fixed work buffers the resident engine will add (delta update, the
            # fp32 MFMA path's hi/lo rows): a shard that fits only without them streams
            delta = cfg.update != "full"
            extra = lloyd_row_extra(cfg.dtype, d, delta)
            fixed = lloyd_fixed_extra(cfg.n_clusters, d, delta, cfg.dtype, xn.shape[0])
            chunk = want or plan_chunk_rows(xn.shape[0], row_bytes, cfg.n_clusters, d, dev,
                                            cfg.hbm_budget_gb, per_row_extra=extra,
                                            extra_fixed=fixed)
            if chunk:
                resident = 0
                if not want:  # planner-driven streaming: keep what fits in HBM resident
                    resident = plan_resident_rows(xn.shape[0], row_bytes, chunk, cfg.n_clusters,
                                                  d, dev, cfg.hbm_budget_gb,
                                                  per_row_extra=lloyd_row_extra(cfg.dtype, d, False))
                return HostSource(xn, layout, dev, row_offset, resident_rows=resident), chunk
        return torch.as_tensor(xn).to(dev), want

    def _build_engine(self, x_local, dev, comm, n_global, row_offset, n_local,
                      init_centers_, start_iter, chunk: int = 0):
        """LloydEngine under the collective OOM agreement (:func:`build_engine_collective`);
        returns (engine, seconds spent creating the data source)."""
        cfg = self.cfg

        def make_engine(source, chunk_rows):
            cls = LloydEngine
            if cfg.algorithm == "bounded":
                from .bounded import BoundedLloydEngine as cls
            return cls(source, cfg, comm, n_global, row_offset, init_centers_, chunk_rows,
                       defer_init=True)

        return build_engine_collective(
            "kmeans", cfg, comm, dev, n_local, start_iter, chunk,
            lambda c: self._make_source(x_local, dev, row_offset, c), make_engine)

    def fit(self, x_local, init_centers_: Optional[np.ndarray] = None,
            n_global: Optional[int] = None, row_offset: Optional[int] = None) -> "KMeans":
        cfg = self.cfg
        t_setup0 = time.perf_counter()
        dev = self._target_device(x_local)
        if self.comm is None:
            self.comm = local_comm(dev)
        comm = self.comm
        n_local = int(x_local.n_rows if hasattr(x_local, "n_rows") else x_local.shape[0])
        if n_global is None or row_offset is None:
            n_global, row_offset = _shard_geometry(n_local, comm)

        ckpt = RunCheckpointer(cfg, comm, "distributedKMeans")
        d = int(x_local.d if hasattr(x_local, "d") else x_local.shape[1])
        resumed = ckpt.load_for_resume(cfg.n_clusters, d)
        start_iter = 0
        if resumed is not None:
            init_centers_, start_iter = resumed.centers, resumed.n_iter
            if comm.is_root:
                print(f"[kmeans] resuming from {cfg.checkpoint_path} at iteration {start_iter}",
                      flush=True)
        eng, initialization_time = self._build_engine(x_local, dev, comm, n_global, row_offset,
                                                      n_local, init_centers_, start_iter)
        if cfg.graph and eng.graphable() and not comm.collective:
            eng.capture()
        if cfg.warmup and cfg.max_iter > eng.n_iter:
            eng.warmup()
        sync(dev)
        # initialization_time: the shard load / H2D (the reference's variable init with the
        # data feed, `:273`); setup_time: the rest (init, kernels' first launch, graph)
        setup_time = time.perf_counter() - t_setup0 - initialization_time

        # ------------------------------------------------------------ timed loop
        history = []
        centers_host = lambda: self.engine_.centers().double().cpu().numpy()
        self.engine_ = eng
        self._retired = []  # weak references to engines replaced after an OOM
        timer = DeviceTimer(dev)
        timer.start()
        while True:
            if eng.oom_guard:
                bad = eng.failed_step(final=eng.n_iter >= cfg.max_iter)
                if bad is not None:
                    # every rank rolls back to the pre-step centroids and continues from the
                    # same iteration on a streamed engine with half the chunk (the reference
                    # restarted the whole run with twice the batches, `:357-360`).  The old
                    # engine (device shard, operand tables, graph pool) is released first.
                    c_host = eng.rollback(bad)
                    n_back, c0 = eng.n_iter, eng.c0
                    chunk = _retry_chunk(eng.chunk_rows, n_local)
                    self._retired.append(weakref.ref(eng))
                    eng = self.engine_ = None
                    _release(dev)
                    if comm.is_root:
                        print(f"[kmeans] out of memory in iteration {n_back + 1}; continuing "
                              f"streamed with chunk_rows={chunk}", flush=True)
                    eng, _ = self._build_engine(x_local, dev, comm, n_global, row_offset, n_local,
                                                c_host, n_back, chunk)
                    eng.c0 = c0
                    self.engine_ = eng
                    continue
            if eng.n_iter >= cfg.max_iter:
                break
            log_pt = cfg.log_every > 0 and (eng.n_iter + 1) % cfg.log_every == 0
            if eng.oom_guard:
                eng.save_state()
            inertia_it = eng.step(with_inertia=log_pt and cfg.compute_inertia)
            if eng.oom_guard:
                eng.post_flag()
            n = eng.n_iter
            if eng.need_shift and (cfg.tol > 0 or log_pt):
                if eng.oom_guard and eng.failed_step(final=True) is not None:
                    continue  # a step failed: recovered at the top of the loop
                sv = float(eng.shift.item())
                rec = {"iter": n, "shift": sv}
                if inertia_it is not None:
                    rec["inertia"] = inertia_it  # of this iteration's assignment (pre-update)
                history.append(rec)
                if log_pt and comm.is_root:
                    extra = f" inertia {inertia_it:.6e}" if inertia_it is not None else ""
                    print(f"[kmeans] iter {n} max centroid shift^2 {sv:.3e}{extra}", flush=True)
                if cfg.tol > 0 and sv <= cfg.tol:
                    break
            if ckpt.due(n):
                if eng.oom_guard and eng.failed_step(final=True) is not None:
                    continue  # never checkpoint centroids of a failed step
                ckpt.maybe_save(n, centers_host)
            faults.maybe_fail(str(n), comm.rank, kinds=("crash",))
        computation_time = timer.stop()
        ckpt.maybe_save(eng.n_iter, centers_host, final=True)

        # ------------------------------------------- final label pass (untimed)
        inertia = eng.label_pass() if cfg.label_pass else None
        n_iter = eng.n_iter
        cnt = eng.exact_counts().cpu().numpy() if n_iter > 0 else None
        self.engine_ = eng
        self.local_ = eng.local
        self.result_ = ClusterResult(
            centers=eng.centers().double().cpu().numpy(), init_centers=eng.c0.cpu().numpy(),
            labels=eng.labels, counts=cnt, n_iter=n_iter, inertia=inertia,
            setup_time=setup_time, initialization_time=initialization_time,
            computation_time=computation_time, backend=eng.local.name, history=history,
            n_global=n_global, streamed=eng.streamed)
        return self

    def predictor(self, device=None):
        """A :class:`..serving.ClusterPredictor` on the fitted centroids (cached per device)."""
        from ..serving import ClusterPredictor
        if self.result_ is None:
            raise RuntimeError("fit() first")
        dev = torch.device(device) if device is not None else torch.device(
            self.result_.labels.device if self.result_.labels is not None else "cpu")
        cache = self.__dict__.setdefault("_predictors", {})
        key = (str(dev), id(self.result_))
        if key not in cache:
            cache.clear()
            cache[key] = ClusterPredictor(self.result_.centers, self.cfg.dtype, dev,
                                          self.cfg.backend)
        return cache[key]

    def predict(self, x: torch.Tensor) -> torch.Tensor:
        """Labels of new points against the fitted centroids (local, no collectives)."""
        x = torch.as_tensor(x)
        return self.predictor(x.device).predict(x)

    def score(self, x: torch.Tensor) -> float:
        """Negative inertia of ``x`` (sklearn convention)."""
        x = torch.as_tensor(x)
        return self.predictor(x.device).score(x)
