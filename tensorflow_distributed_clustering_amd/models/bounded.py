"""Exact Lloyd iterations with bounds-based pruning (``ClusterConfig(algorithm="bounded")``).

Hamerly (2010)'s single-lower-bound form of Lloyd, on the MI355X kernels: each row keeps
an upper bound ``ub`` on the distance to its centroid and a lower bound ``lb`` on the
distance to every other centroid.  After the centroids move by ``drift[k]``,
``ub += drift[a]`` and ``lb -= max(drift)``; a row with ``ub < lb`` provably keeps its
label (same argmin as a full Lloyd assignment), so only the remaining rows are
re-assigned, by the indexed top-2 MFMA kernel (which also refreshes both bounds), and
only the rows whose label changed move their contribution between the per-cluster
totals (two indexed counting-sort updates: +x into the new cluster, -x out of the old).
The totals are fp64 and replicated on every rank; the per-iteration DELTAS go through
ONE packed all-reduce, exactly like the Lloyd partials.

The reference has only plain Lloyd (`scripts/distribuitedClustering.py:180-294`); this is
an opt-in algorithm with the same fixed points.  Results equal Lloyd's up to bf16
near-ties (``slack`` widens the bound test by that relative margin) and fp32 summation
order; the totals are recomputed from scratch every ``refresh`` (64) iterations.

Requirements: the resident bf16 MFMA path (D <= 256) with the sorted update (K x D past
the LDS-privatised update); other configurations run plain Lloyd (``LloydEngine``).
"""
from __future__ import annotations

from typing import Optional

import torch

from .kmeans import LloydEngine


def bounded_supported(eng: LloydEngine) -> bool:
    sup = getattr(eng.local, "supports_indexed", None)
    return (eng.device.type == "cuda" and not eng.streamed and sup is not None and sup()
            and hasattr(eng.local.ops, "assign_bf16_top2")
            and eng.cfg.empty_cluster in ("keep", "nan", "zero", "reseed"))


class BoundedLloydEngine(LloydEngine):
    """LloydEngine whose ``step()`` re-assigns only the rows the bounds cannot settle."""

    # the totals are fp64 (gbuf) and the per-step deltas small: plain [sums | counts] buffer
    exact_counts_ok = False
    delta_ok = False  # its own moved-row bookkeeping (bounds_scatter)
    fixed_ok = False  # float delta arithmetic on buf (deterministic: plain Lloyd steps)
    rsag_ok = False
    warmup_ok = False  # the bounds and running totals are incremental
    oom_guard_ok = False
    slack = 1e-3     # relative margin on ub (bf16 distance arithmetic)
    refresh = 64     # iterations between full recomputations of the totals

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.enabled = bounded_supported(self)  # else: plain Lloyd steps
        self.active_frac = 1.0
        if not self.enabled:
            return
        n, k, d, dev = self.n_local, self.k, self.d, self.device
        self.ub = torch.zeros(n, dtype=torch.float32, device=dev)
        self.lb = torch.zeros(n, dtype=torch.float32, device=dev)
        self.d1 = torch.zeros(n, dtype=torch.float32, device=dev)
        self.d2 = torch.zeros(n, dtype=torch.float32, device=dev)
        self.active = torch.zeros(n, dtype=torch.int32, device=dev)
        self.blab = torch.zeros(n, dtype=torch.int32, device=dev)
        self.moved = torch.zeros(3, n, dtype=torch.int32, device=dev)  # idx | old | new
        self.cnt = torch.zeros(2, dtype=torch.int32, device=dev)       # active | moved
        self.minus = torch.zeros_like(self.buf)
        # fp64 running totals, laid out like buf[:k*d+k] so one kernel updates both
        self.gbuf = torch.zeros(k * d + k, dtype=torch.float64, device=dev)
        self.gsums = self.gbuf[: k * d].view(k, d)
        self.gcounts = self.gbuf[k * d:]
        self.drift = torch.zeros(k, dtype=torch.float32, device=dev)
        self.maxdrift = torch.zeros(1, dtype=torch.float32, device=dev)
        self._fresh = True       # next step is a full assignment (first step / refresh)

    def rewind(self, snap: dict):
        super().rewind(snap)
        if self.enabled:
            self._fresh = True  # bounds and totals are rebuilt by a full top-2 pass

    def graphable(self) -> bool:
        # data-dependent launch sizes (the host reads the active / moved counts)
        return False if self.enabled else super().graphable()

    # --------------------------------------------------------------------- steps
    def _eager_step(self, with_inertia: bool = False) -> Optional[float]:
        if not self.enabled:
            return super()._eager_step(with_inertia)
        lo, ops, x = self.local, self.local.ops, self.local.x
        C_prev = self.C.clone() if (self.cfg.spherical or self.cfg.empty_cluster == "reseed") \
            else None
        k, d = self.k, self.d
        inertia = None
        if self._fresh or with_inertia or (self.n_iter % self.refresh == 0):
            # full top-2 assignment: labels, exact distances, both bounds; totals from
            # scratch (the Lloyd partials of this assignment)
            ops.assign_bf16_top2(x, None, lo.cm2, lo.cnorm, self.labels, self.d1, self.d2)
            torch.sqrt(self.d1, out=self.ub)
            torch.sqrt(self.d2, out=self.lb)
            self.buf.zero_()
            lo.update(x, self.labels, self.sums, self.counts)
            if with_inertia:
                inertia = self.comm.sum_scalar(float(self.d1.double().sum()))
            self.comm.allreduce_bucketed_(self.buf, self.bucket_bytes)
            self.gbuf.copy_(self.buf[: self.gbuf.numel()])
            self.active_frac = 1.0
            self._fresh = False
        else:
            self.cnt.zero_()
            ops.bounds_filter(self.labels, self.ub, self.lb, self.drift, self.maxdrift,
                              self.slack, self.active, self.cnt[0:1])
            self.buf.zero_()  # queued ahead of the host read of the active count
            self.minus.zero_()
            m = int(self.cnt[0].item())
            if m > 0:
                act = self.active[:m]
                ops.assign_bf16_top2(x, act, lo.cm2, lo.cnorm, self.blab[:m], self.d1[:m],
                                     self.d2[:m])
                ops.bounds_scatter(act, self.cnt[0:1], self.blab[:m], self.d1[:m], self.d2[:m],
                                   self.labels, self.ub, self.lb, self.moved[0, :m],
                                   self.moved[1, :m], self.moved[2, :m], self.cnt[1:2])
                mv = int(self.cnt[1].item())
                if mv > 0:
                    idx = self.moved[0, :mv]
                    lo.update.indexed(x, idx, self.moved[2, :mv], self.sums, self.counts)
                    ms = self.minus[: k * d].view(k, d)
                    mc = self.minus[k * d: k * d + k]
                    lo.update.indexed(x, idx, self.moved[1, :mv], ms, mc)
            self.active_frac = m / max(1, self.n_local)
            self.buf.sub_(self.minus)  # deltas: +x into new clusters, -x out of old ones
            self.comm.allreduce_bucketed_(self.buf, self.bucket_bytes)
            self.gbuf.add_(self.buf[: self.gbuf.numel()])
        if self.shift is not None:
            self.shift.zero_()
        moved_after = self.cfg.spherical or self.cfg.empty_cluster == "reseed"
        if not moved_after:
            # the finalize kernel also emits each centroid's movement (bf16 coordinates,
            # NaN stays NaN -> every row re-assigned) and its max
            self.maxdrift.zero_()
            lo.ops.finalize(self.gsums, self.gcounts, self.C, lo.policy, self.shift, lo.cm2,
                            lo.cnorm, self.drift, self.maxdrift)
        else:
            lo.ops.finalize(self.gsums, self.gcounts, self.C, lo.policy, self.shift, lo.cm2,
                            lo.cnorm)
            if self.cfg.spherical:
                self.C.div_(self.C.norm(dim=1, keepdim=True).clamp_min_(1e-30))
                lo.prepare(self.C)
            if self.cfg.empty_cluster == "reseed":
                # _reseed() reads self.counts: give it the totals of the current
                # assignment, not this step's all-reduced deltas
                self.counts.copy_(self.gcounts)
                self._reseed()
            # centroid drift in the kernels' own (bf16-rounded) centroid coordinates
            dc = self.C.to(torch.bfloat16).float() - C_prev.to(torch.bfloat16).float()
            torch.linalg.vector_norm(dc, dim=1, out=self.drift)
            torch.nan_to_num_(self.drift, nan=float("inf"))
            torch.amax(self.drift, dim=0, keepdim=True, out=self.maxdrift)
        # counts of the current assignment (ClusterResult.counts)
        self.counts.copy_(self.gcounts)
        self.n_iter += 1
        return inertia
