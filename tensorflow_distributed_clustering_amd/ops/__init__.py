"""Op layer: the local (per-rank) part of one clustering iteration.

Each *local-ops* object owns the shard in the layout its kernels want and exposes
three calls used by the algorithm drivers in :mod:`..models`:

``step(C, labels, mind, sums, counts)``   assignment + per-cluster partials
``assign(C, labels, mind)``               label pass only (reference `:282`)
``finalize(sums, counts, C, policy, shift)`` centroid divide (+ operand prep)

Variants (picked by :func:`make_lloyd_ops`):

========================  =====================================================
``HipBf16Lloyd``          bf16 MFMA distance+argmin (N1) + LDS update (N2) + N3
``HipWideBf16Lloyd``      bf16, 256 < D <= 1024: K-grouped wide-D MFMA kernel
``HipFp8Lloyd``           fp8 e4m3 + E8M0 block scales (N8), scaled-MFMA assign,
                          update from the full-precision shard
``HipSmallLloyd``         fused fp32/fp64 assign+accumulate (reference configs)
``HipSimtLloyd``          fp32/fp64 exact SIMT assign + LDS update
``HipX3Lloyd``            fp32/fp64, 16 < D <= 1024: bf16x3 MFMA scores + top-3, exact
                          re-check of the rows the error bound cannot certify
``HipExactLloyd``         fp32/fp64 D > 1024 (and bf16 D > 1024), or exact_assign='simt':
                          tiled exact difference-form assign
``TorchLloyd``            plain PyTorch (CPU ranks, oracle)
========================  =====================================================
"""
from __future__ import annotations

from typing import Optional

import torch

from .. import _native
from ..parallel.dist import join_counts, split_counts
from . import reference as ref

POLICY_CODES = {"keep": 0, "reseed": 0, "nan": 1, "nan_any": 1, "zero": 2}
TORCH_DTYPES = {"fp64": torch.float64, "fp32": torch.float32, "bf16": torch.bfloat16,
                "fp8": torch.bfloat16}
MFMA_DIMS = (32, 64, 128, 256)
WIDE_BF16_DIMS = (384, 512, 640, 768, 896, 1024)
FP8_DIMS = (256, 512, 768, 1024)


def acc_dtype_for(dtype: str, k: int, d: int) -> torch.dtype:
    """Accumulation / all-reduce dtype of the per-cluster partials.

    fp64 whenever the buffer is small (latency-bound all-reduce: the extra bytes are
    free and counts stay exact past 2^24); fp32 for big K x D buffers.
    """
    if dtype == "fp64" or k * (d + 1) <= 65536:
        return torch.float64
    return torch.float32


def padded_dim(d: int) -> Optional[int]:
    for p in MFMA_DIMS:
        if d <= p:
            return p
    return None


def wide_bf16_dim(d: int) -> Optional[int]:
    for p in WIDE_BF16_DIMS:
        if d <= p:
            return p
    return None


def fp8_dim(d: int) -> Optional[int]:
    for p in FP8_DIMS:
        if d <= p:
            return p
    return None


# work items (point block x K-group) the wide-D kernel needs to fill 256 CUs
KGROUP_MIN_ITEMS = 2048


def kgroup_tiles(row_bytes: int, kp: int, n: Optional[int] = None,
                 group_bytes: int = 0) -> int:
    """Centroid tiles (of 32) per K-group (0 = one group over all of K).

    ``group_bytes`` > 0 (``ClusterConfig.kgroup_bytes``): groups of that many centroid
    bytes, for L2 residency per XCD.  Measured slower than one group (the 256 MiB MALL
    serves the 48 MiB fp8 table: N=5M D=768 K=65536, 3 MiB groups 206.5 ms vs one group
    197.3 ms, docs/PERF_NOTES.md), so the default is 0.  Otherwise one group, unless the
    point count is too small to fill the chip (serving requests, small chunks): then K is
    split so that (N/256 point blocks) x groups reaches KGROUP_MIN_ITEMS work items (1024
    rows x K=65536 fp8: 4 items -> 2.2 ms; the groups' winners merge through the 64-bit
    key atomics).  Groups are a whole number of 64-row stages."""
    ntiles = kp // 32
    if group_bytes > 0:
        tiles = max(1, group_bytes // (32 * row_bytes))
        return 0 if tiles * 32 >= kp else int(tiles)
    if n is None:
        return 0
    npb = max(1, (n + 255) // 256)
    if npb >= KGROUP_MIN_ITEMS or ntiles < 4:
        return 0
    groups = min(-(-KGROUP_MIN_ITEMS // npb), ntiles // 2)
    tiles = -(-ntiles // groups)
    tiles += tiles & 1
    return 0 if tiles >= ntiles else int(tiles)


def use_native(device: torch.device, backend: str) -> bool:
    if backend == "torch" or device.type != "cuda":
        if backend == "hip" and device.type != "cuda":
            raise RuntimeError("backend='hip' requires a GPU tensor")
        return False
    _native.require()  # GPU + hip/auto: the native path is mandatory (fail loudly)
    return True


class NativeUpdate:
    """N2 dispatcher: LDS-privatised histogram when K x D fits one LDS slice, otherwise
    counting sort + segmented gather-sum (workspace allocated once per shard).

    ``deterministic`` (ClusterConfig.deterministic): the sorted path with
    FIXED-POINT partials -- every element is rounded toward zero to an int64 multiple of
    2^-S (``fixed_scale`` = 2^S, chosen by the engine from the global max |x| and N so no
    sum can overflow) and summed in int64.  Integer addition is associative, so the float
    atomics' arrival order no longer matters: the update, the int64 all-reduce and the
    finalize are bitwise reproducible run to run and across world sizes.  Callers with
    float buffers (mini-batches) get the fixed-point sums converted back."""

    LDS_BUDGET = 64 * 1024

    def __init__(self, ops, n: int, k: int, d: int, x_dtype: torch.dtype, device,
                 deterministic: bool = False):
        self.ops = ops
        self.deterministic = bool(deterministic)
        es = 8 if x_dtype == torch.float64 else 4
        self.kind = "lds" if k * (d + 1) * es + 4 * k <= self.LDS_BUDGET else "sorted"
        if self.deterministic:
            self.kind = "sorted"
        self.work = None
        self._fx = None
        if self.kind == "sorted":
            self.work = self._workspace(n, k, device)

    @staticmethod
    def _workspace(n, k, device):
        # zero-filled once: the kernels leave its histogram part zeroed after every call
        return torch.zeros(int(_native.require().update_sorted_workspace(n, k)),
                           dtype=torch.int32, device=device)

    # 2^S of the fixed-point partials (deterministic); set by the engine before the first step
    fixed_scale = 0.0
    # (hi, lo) fp32 [K] views of the all-reduce buffer: exact count halves
    # (parallel/dist.split_counts), accumulated by the scan kernel of the sorted update
    count_split = None
    # the engine's all-reduce buffer when the step's zero fill rides in the first update
    # kernel (resident sorted path); consumed by the next call only
    zero_buf = None

    def fuses_zero(self) -> bool:
        return self.kind == "sorted"

    def __call__(self, x, labels, sums, counts):
        if self.kind == "lds":
            self.ops.update(x, labels, sums, counts)
            if self.count_split is not None:
                split_counts(torch.bincount(labels[: x.shape[0]].long(), minlength=sums.shape[0]),
                             *self.count_split)
            return
        if self.work.numel() < int(self.ops.update_sorted_workspace(x.shape[0], sums.shape[0])):
            self.work = self._workspace(x.shape[0], sums.shape[0], x.device)
        if self.deterministic and sums.dtype != torch.int64:
            self._fixed_into_float(x, labels, sums, counts)
            return
        # work_clean: the workspace was zero-filled when allocated and every call leaves
        # its histogram zeroed (no memset launch per step)
        self.ops.update_sorted(x, labels, sums, counts, self.work, *(self.count_split or (None, None)),
                               self.zero_buf, self.fixed_scale if sums.dtype == torch.int64 else 0.0,
                               True)

    def _fixed_into_float(self, x, labels, sums, counts):
        """Deterministic partials for a float buffer: fixed-point into an int64 scratch
        (scale from this call's rows), then added to the caller's buffer."""
        k, d = sums.shape
        if self._fx is None or self._fx.numel() != k * d + k:
            self._fx = torch.zeros(k * d + k, dtype=torch.int64, device=x.device)
        self._fx.zero_()
        n = x.shape[0]
        scale = fixed_point_scale(float(x[:, :d].abs().max()) if n else 0.0, n,
                                  elem32=x.dtype != torch.float64)
        fs, fc = self._fx[: k * d].view(k, d), self._fx[k * d:]
        self.ops.update_sorted(x, labels, fs, fc, self.work, None, None, None, scale, True)
        sums.add_((fs.double() / scale).to(sums.dtype))
        counts.add_(fc.to(counts.dtype))
        if self.count_split is not None:
            split_counts(fc, *self.count_split)


    def supports_indexed(self) -> bool:
        return self.kind == "sorted" and not self.deterministic

    def indexed(self, x, rowidx, labels, sums, counts, zero_first=None):
        """Partials of the rows ``x[rowidx]`` without gathering them (mini-batches).
        ``zero_first``: a buffer (the step's all-reduce buffer, holding sums / counts) the
        first update kernel clears before anything accumulates into it."""
        need = int(self.ops.update_sorted_workspace(rowidx.shape[0], sums.shape[0]))
        if self.work is None or self.work.numel() < need:
            self.work = self._workspace(rowidx.shape[0], sums.shape[0], x.device)
        self.ops.update_sorted_indexed(x, rowidx, labels, sums, counts, self.work,
                                       *(self.count_split or (None, None)), True, zero_first)


# ----------------------------------------------------------------- delta update
# ctrl words (csrc/kernels.h TdcDeltaCtrl)
DC_NEXT, DC_MODE, DC_MOVED, DC_EVENTS, DC_PREVOK, DC_ITER, DC_WORDS = 0, 1, 2, 3, 4, 5, 16
DELTA_MAX_K = 65536


class DeltaState:
    """Running state of the delta centroid update of plain Lloyd (ClusterConfig.update).

    Invariant: ``G = [sums K*D | counts K]`` (fp64, replicated on every rank) are the
    per-cluster totals of the assignment held in ``prev`` (the previous step's labels on
    every rank).  A *delta* step sums only the rows whose label changed, +x into the new
    and -x out of the old cluster, into the step's all-reduce buffer; the finalize adds
    the all-reduced deltas to G and divides.  A *full* step sums every row and replaces G.
    The mode of each step lives in ``ctrl`` on the device: the previous finalize picks it
    from the all-reduced moved count (the same on every rank), so the step needs no host
    sync and stays capturable.  Full steps: the first one after :meth:`reset`, every
    ``refresh`` steps, and after a step that moved more than ``theta`` of all rows.

    The reference re-summed every row every iteration (K Where/Gather chains + a CPU
    bincount, `scripts/distribuitedClustering.py:237-263`); the fixed points are the same.
    """

    def __init__(self, n: int, k: int, d: int, device, refresh: int, theta: float,
                 g_rows: Optional[int] = None):
        self.n, self.k, self.d = n, k, d
        # rows of the replicated totals this rank keeps: all K, or (reduce-scatter mode) the
        # rank's own slice of centroid rows
        self.gk = k if g_rows is None else int(g_rows)
        self.refresh, self.theta = int(refresh), float(theta)
        self.prev = torch.zeros(max(1, n), dtype=torch.int32, device=device)
        self.G = torch.zeros(self.gk * d + self.gk, dtype=torch.float64, device=device)
        self.ctrl = torch.zeros(DC_WORDS, dtype=torch.int32, device=device)
        # [moved rows (steps with a valid prev), such steps, full steps, steps]
        self.stats = torch.zeros(4, dtype=torch.float64, device=device)
        self.reset()

    @property
    def sums(self) -> torch.Tensor:
        return self.G[: self.gk * self.d].view(self.gk, self.d)

    @property
    def counts(self) -> torch.Tensor:
        return self.G[self.gk * self.d:]

    def reset(self):
        """The next step is a full one and ``prev`` holds no labels yet (after the centroid
        init, or anything else that breaks the invariant)."""
        self.ctrl.zero_()
        self.ctrl[DC_NEXT] = 1

    def stats_host(self) -> dict:
        v = self.stats.tolist()
        return {"moved_rows": v[0], "moved_steps": v[1], "full_steps": v[2], "steps": v[3]}


class NativeDelta(DeltaState):
    """HIP delta update (csrc/update_sorted.hip delta_*, centroids.hip finalize_delta).
    With int64 buffers (the deterministic update) the deltas are fixed point
    (``fixed_scale``, set by the engine) and exactly reproducible."""
    native = True
    fixed_scale = 0.0

    def __init__(self, ops, n, k, d, device, refresh, theta, g_rows=None):
        super().__init__(n, k, d, device, refresh, theta, g_rows)
        self.ops = ops
        self.work = torch.zeros(int(ops.delta_workspace(n, k)), dtype=torch.int32, device=device)

    def update(self, x, labels, sums, counts, split, moved, zero_buf):
        hi, lo = split or (None, None)
        fx = self.fixed_scale if sums.dtype == torch.int64 else 0.0
        self.ops.delta_update(x, labels, self.prev, sums, counts, self.work, self.ctrl, hi, lo,
                              moved, zero_buf, fx, True)

    def finalize(self, sums, counts, split, moved, C, policy, shift, cm2, cnorm, n_global):
        hi, lo = split or (None, None)
        fx = self.fixed_scale if sums.dtype == torch.int64 else 0.0
        self.ops.delta_finalize(sums.reshape(-1), counts, hi, lo, moved, self.G, C, policy, shift,
                                cm2, cnorm, self.ctrl, self.stats, self.refresh,
                                self.theta * float(n_global), fx)


class TorchDelta(DeltaState):
    """The same state machine in PyTorch ops (CPU ranks over gloo, ``backend='torch'``)."""
    native = False

    def __init__(self, n, k, d, device, refresh, theta, empty_cluster="keep", g_rows=None):
        super().__init__(n, k, d, device, refresh, theta, g_rows)
        self.empty_cluster = empty_cluster

    def update(self, x, labels, sums, counts, split, moved, zero_buf):
        full = bool(self.ctrl[DC_NEXT])
        n, k, d = x.shape[0], self.k, sums.shape[1]
        new = labels[:n].long()
        old = self.prev[:n].long()
        mv = new != old
        xs = x[:, :d].to(sums.dtype)
        if full:
            sums.index_add_(0, new, xs)
            c = torch.bincount(new, minlength=k)
        else:
            idx = torch.nonzero(mv).flatten()
            sums.index_add_(0, new[idx], xs[idx])
            sums.index_add_(0, old[idx], -xs[idx])
            c = torch.bincount(new[idx], minlength=k) - torch.bincount(old[idx], minlength=k)
        counts.add_(c.to(counts.dtype))
        if split is not None:
            split_counts(c, *split)
        self.prev[:n].copy_(labels[:n])
        if moved is not None:
            moved.add_(mv.sum().to(moved.dtype))
        self.ctrl[DC_MODE] = int(full)

    def finalize(self, sums, counts, split, moved, C, policy, shift, cm2, cnorm, n_global):
        full = bool(self.ctrl[DC_MODE])
        dc = join_counts(*split) if split is not None else counts.double()
        if full:
            self.G.zero_()
        self.sums.add_(sums.double())
        self.counts.add_(dc)
        new = ref.finalize(self.sums, self.counts, C, self.empty_cluster)
        if shift is not None:
            dd = new.double() - C.double()
            shift.fill_(float((dd * dd).sum(1).max()) if dd.numel() else 0.0)
        C.copy_(new)
        it = int(self.ctrl[DC_ITER]) + 1
        prev_ok = bool(self.ctrl[DC_PREVOK])
        m = float(moved) if moved is not None else 0.0
        nxt = (self.refresh > 0 and it % self.refresh == 0) or \
              (prev_ok and m > self.theta * float(n_global))
        self.ctrl[DC_ITER] = it
        self.ctrl[DC_NEXT] = int(nxt)
        self.ctrl[DC_PREVOK] = 1
        self.stats += torch.tensor([m if prev_ok else 0.0, float(prev_ok), float(full), 1.0],
                                   dtype=torch.float64, device=self.stats.device)


def fixed_point_scale(max_abs: float, n_rows: int, elem32: bool = True) -> float:
    """2^S for fixed-point partial sums of up to ``n_rows`` values of magnitude <=
    ``max_abs``: the largest power of two with max_abs * n_rows * 2^S < 2^61 (no int64 sum
    can overflow) and, with ``elem32`` (bf16 / fp32 rows), max_abs * 2^S <= 2^30 (every
    element's fixed point fits an int32: the kernels round it with one v_rndne + v_cvt_i32
    instead of the emulated float -> int64 conversion), clamped to [2^-60, 2^60].  The
    step 2^-S is then max_abs * 2^-30 or finer -- below the fp32 ulp of the largest
    element; fp64 rows (``elem32=False``) get the finer step the sum bound allows.  The
    kernels round to nearest (unbiased)."""
    import math
    m = float(max_abs)
    if not math.isfinite(m):
        raise ValueError("deterministic update: the data holds a NaN or an infinity "
                         "(no fixed-point scale exists for non-finite values)")
    m = max(m, 1e-30)
    s_sum = math.floor(61 - math.log2(m * max(1, int(n_rows)))) - 1
    s_elem = math.floor(30 - math.log2(m)) if elem32 else s_sum
    return float(2.0 ** max(-60, min(60, s_sum, s_elem)))


class _LocalOpsBase:
    name = "base"

    def __init__(self, x: torch.Tensor, k: int, empty_cluster: str = "keep"):
        self.n, self.d = x.shape
        self.k = k
        self.device = x.device
        self.policy = POLICY_CODES[empty_cluster]
        self.empty_cluster = empty_cluster

    # centroid dtype kept by the driver
    c_dtype = torch.float32
    # 2^S of fixed-point (int64) partial sums -- the deterministic update; 0: float sums
    fixed_scale = 0.0

    def set_fixed_scale(self, scale: float):
        self.fixed_scale = float(scale)
        upd = getattr(self, "update", None)
        if isinstance(upd, NativeUpdate):
            upd.fixed_scale = float(scale)

    def fixed_point(self) -> bool:
        """Deterministic partials in int64 fixed point (native update, deterministic)."""
        upd = getattr(self, "update", None)
        return isinstance(upd, NativeUpdate) and upd.deterministic

    @property
    def layout(self):
        """(dtype, width) of the row layout the kernels consume (for chunk sources)."""
        return (self.x.dtype, self.x.shape[1])

    def bind(self, x: torch.Tensor):
        """Point the kernels at another chunk already in :attr:`layout` (streaming)."""
        if x.dtype != self.x.dtype or x.shape[1] != self.x.shape[1]:
            raise ValueError(f"chunk layout {(x.dtype, x.shape[1])} != {self.layout}")
        self.x = x
        self.n = x.shape[0]
        return self

    def unbind(self):
        """Drop the reference to the last streamed chunk: it is a view of the source's
        device slot, which would otherwise stay allocated next to the next pass's slots."""
        x = getattr(self, "x", None)
        if isinstance(x, torch.Tensor) and x.numel():
            self.x = x.new_empty((0,) + tuple(x.shape[1:]))
            self.n = 0

    def prepare(self, C: torch.Tensor):
        """(Re)derive kernel operands from C (called after init / external edits)."""

    def finalize(self, sums, counts, C, shift):
        ref_new = ref.finalize(sums, counts, C, self.empty_cluster)
        if shift is not None:
            d = (ref_new.double() - C.double())
            shift.fill_(float((d * d).sum(1).max()) if d.numel() else 0.0)
        C.copy_(ref_new)
        self.prepare(C)

    # ------------------------------------------ reduce-scatter / all-gather (rsag) mode
    # centroid-row multiple the assign operands need (MFMA tiles)
    row_align = 1

    def pad_rows(self, kpad: int):
        """Give the assign operands ``kpad`` centroid rows (rsag: one equal slice per rank)."""

    def gather_operands(self):
        """Tensors (dim 0 = centroid rows, ``kpad`` of them) the assignment reads; the
        rsag engine all-gathers these after each rank prepped its slice.  None: the
        assignment reads the fp32/fp64 centroids themselves."""
        return None

    def finalize_rows(self, sums, counts, C, shift, r0: int, kr: int):
        """Finalize the centroid rows ``C`` (= rows [r0, r0 + len(C)) of the full table) and
        prep operand rows [r0, r0 + kr) (rows past K become padding).  ``shift`` (if given)
        is raised to this slice's max shift^2."""
        if C.shape[0] == 0:
            return
        new = ref.finalize(sums, counts, C, self.empty_cluster)
        if shift is not None:
            d = new.double() - C.double()
            shift.fill_(max(float(shift.max()), float((d * d).sum(1).max())))
        C.copy_(new)

    # ------------------------------------------------------------- delta update
    def make_delta(self, n: int, k: int, d: int, refresh: int, theta: float,
                   empty_cluster: str = "keep", g_rows: Optional[int] = None):
        """A :class:`DeltaState` for this shard, or None where the delta update is not
        supported (fused assign+update kernels, K > 65536, shards of 2^30 rows or more).
        ``g_rows``: rows of the totals this rank keeps (reduce-scatter mode: its slice)."""
        upd = getattr(self, "update", None)
        if not isinstance(upd, NativeUpdate) or k > DELTA_MAX_K:
            return None
        if n >= (1 << 30):
            return None
        return NativeDelta(self.ops, n, k, d, self.device, refresh, theta, g_rows)

    def prep_rows(self, C: torch.Tensor, r0: int, kr: int):
        """rsag: the assign-operand rows [r0, r0 + kr) from the finalised centroid slice C
        (rows past K become padding); no-op where the ranks gather the centroids."""

    def bf16_operands(self):
        """(Cm2, cnorm) the finalize kernel writes for the next assignment, or (None, None)."""
        return None, None

    def after_finalize(self, C: torch.Tensor):
        """Operand prep the finalize kernel does not do itself (fp8 re-quantisation)."""

    def after_gather(self, C: torch.Tensor):
        """rsag: operand prep after the all-gather, when :meth:`gather_operands` is None
        (the ranks gathered the centroids themselves)."""

    # ------------------------------------------------------------- exact counts
    def supports_count_split(self) -> bool:
        return isinstance(getattr(self, "update", None), NativeUpdate)

    def set_count_split(self, hi, lo):
        self.update.count_split = (hi, lo)


class TorchLloyd(_LocalOpsBase):
    name = "torch"

    def __init__(self, x, k, dtype="fp64", empty_cluster="keep", exact=None):
        super().__init__(x, k, empty_cluster)
        tdt = TORCH_DTYPES[dtype] if dtype in ("fp64", "fp32") else torch.float32
        self.x = x.to(tdt).contiguous()
        self.c_dtype = tdt
        self.exact = (dtype == "fp64") if exact is None else exact

    count_split = None

    def supports_count_split(self) -> bool:
        return True

    def set_count_split(self, hi, lo):
        self.count_split = (hi, lo)

    def step(self, C, labels, mind, sums, counts):
        lab, md = ref.assign(self.x, C.to(self.x.dtype), exact=self.exact)
        labels.copy_(lab)
        if mind is not None:
            mind.copy_(md)
        s, c = ref.cluster_sums(self.x, lab, self.k, acc_dtype=sums.dtype)
        sums.add_(s)
        counts.add_(c)
        if self.count_split is not None:
            split_counts(torch.bincount(lab.long(), minlength=self.k), *self.count_split)

    def assign(self, C, labels, mind):
        lab, md = ref.assign(self.x, C.to(self.x.dtype), exact=self.exact)
        labels.copy_(lab)
        if mind is not None:
            mind.copy_(md)

    def make_delta(self, n, k, d, refresh, theta, empty_cluster="keep", g_rows=None):
        return TorchDelta(n, k, d, self.device, refresh, theta, empty_cluster, g_rows)


class HipBf16Lloyd(_LocalOpsBase):
    """bf16 shard [N, DP] (zero-padded to an MFMA-friendly width) + fp32 centroids."""
    name = "hip_bf16_mfma"
    c_dtype = torch.float32

    def __init__(self, x, k, empty_cluster="keep"):
        super().__init__(x, k, empty_cluster)
        self.ops = _native.require()
        dp = padded_dim(self.d)
        if dp is None:
            raise ValueError(f"bf16 MFMA path supports D <= {MFMA_DIMS[-1]}, got {self.d}")
        self.dp = dp
        if x.dtype == torch.bfloat16 and self.d == dp and x.is_contiguous():
            self.x = x
        else:
            xb = torch.zeros(self.n, dp, dtype=torch.bfloat16, device=x.device)
            xb[:, : self.d] = x
            self.x = xb
        self.kp = ((k + 63) // 64) * 64
        self.cm2 = torch.zeros(self.kp, dp, dtype=torch.bfloat16, device=x.device)
        self.cnorm = torch.zeros(self.kp, dtype=torch.float32, device=x.device)
        self.update = NativeUpdate(self.ops, self.n, k, self.d, torch.bfloat16, x.device)

    def prepare(self, C):
        self.ops.finalize(None, None, C, 0, None, self.cm2, self.cnorm)

    def step(self, C, labels, mind, sums, counts):
        self.ops.assign_bf16(self.x, self.cm2, self.cnorm, labels, mind)
        self.update(self.x, labels, sums, counts)

    def assign(self, C, labels, mind):
        self.ops.assign_bf16(self.x, self.cm2, self.cnorm, labels, mind)

    def finalize(self, sums, counts, C, shift):
        self.ops.finalize(sums, counts, C, self.policy, shift, self.cm2, self.cnorm,
                          fixed_scale=self.fixed_scale)

    def bf16_operands(self):
        return self.cm2, self.cnorm

    # -------------------------------------------------- mini-batches by row index
    def supports_indexed(self) -> bool:
        return self.dp in (64, 128, 256) and self.update.supports_indexed()

    def step_indexed(self, C, rowidx, labels, mind, sums, counts, zero_first=None):
        """Assign + partials of the shard rows ``rowidx`` (int32 [B]); the batch is never
        copied out of the shard (the kernels load row rowidx[i] for point i).
        ``zero_first``: see NativeUpdate.indexed (sums / counts need no clearing then)."""
        self.ops.assign_bf16_indexed(self.x, rowidx, self.cm2, self.cnorm, labels, mind)
        self.update.indexed(self.x, rowidx, labels, sums, counts, zero_first)

    def sculley(self, sums, counts, C, v, shift):
        """Native mini-batch centre update + next-assignment operand prep (one launch)."""
        self.ops.sculley_update(sums, counts, C, v, shift, self.cm2, self.cnorm)

    row_align = 64

    def pad_rows(self, kpad):
        if kpad != self.kp:
            self.kp = kpad
            self.cm2 = torch.zeros(kpad, self.dp, dtype=torch.bfloat16, device=self.device)
            self.cnorm = torch.zeros(kpad, dtype=torch.float32, device=self.device)

    def gather_operands(self):
        return [self.cm2, self.cnorm]

    def finalize_rows(self, sums, counts, C, shift, r0, kr):
        self.ops.finalize(sums, counts, C, self.policy, shift, self.cm2[r0:r0 + kr],
                          self.cnorm[r0:r0 + kr], fixed_scale=self.fixed_scale)

    def prep_rows(self, C, r0, kr):
        self.ops.finalize(None, None, C, 0, None, self.cm2[r0:r0 + kr], self.cnorm[r0:r0 + kr])


class _GroupedAssign:
    """Shared state of the K-grouped wide-D kernels: point norms + merge keys."""

    # ClusterConfig.kgroup_bytes (0: one K-group unless the launch is too small to fill
    # the chip); set by the engine after construction
    kgroup_bytes = 0

    def _init_grouped(self, row_bytes: int):
        self._row_bytes = row_bytes
        self.kg = kgroup_tiles(row_bytes, self.kp, group_bytes=self.kgroup_bytes)
        self._keys = None

    def _kg_for(self, n: int) -> int:
        """K-group size for an n-row launch (splits K when n alone cannot fill the chip)."""
        self.kg = kgroup_tiles(self._row_bytes, self.kp, n, self.kgroup_bytes)
        return self.kg

    def _keys_for(self, n):
        if self.kg == 0:
            return None
        if self._keys is None or self._keys.numel() < n:
            self._keys = torch.full((max(n, 1),), -1, dtype=torch.int64, device=self.device)
        return self._keys[:n]


class HipWideBf16Lloyd(_GroupedAssign, _LocalOpsBase):
    """bf16 shard [N, DP], 256 < D <= 1024 (DP = 384 ... 1024 in steps of 128): assign_bigd
    bf16 kernel (8-wave groups up to 512, one wave per SIMD above: the point fragments are
    D/4 registers)."""
    name = "hip_bf16_wide"
    c_dtype = torch.float32

    def __init__(self, x, k, empty_cluster="keep"):
        super().__init__(x, k, empty_cluster)
        self.ops = _native.require()
        self.dp = wide_bf16_dim(self.d)
        if self.dp is None:
            raise ValueError(f"wide bf16 path supports D <= {WIDE_BF16_DIMS[-1]}, got {self.d}")
        self.x = None
        self.kp = ((k + 31) // 32) * 32
        self.cm2 = torch.zeros(self.kp, self.dp, dtype=torch.bfloat16, device=x.device)
        self.cnorm = torch.zeros(self.kp, dtype=torch.float32, device=x.device)
        self._init_grouped(self.dp * 2 + 4)
        self._set_x(x)
        self.update = NativeUpdate(self.ops, self.n, k, self.d, torch.bfloat16, x.device)

    def _set_x(self, x):
        if x.dtype == torch.bfloat16 and x.shape[1] == self.dp and x.is_contiguous():
            xb = x
        else:
            xb = torch.zeros(x.shape[0], self.dp, dtype=torch.bfloat16, device=x.device)
            xb[:, : min(self.d, x.shape[1])] = x[:, : self.d]
        self.x = xb
        self.n = xb.shape[0]
        self.xnorm = xb.float().pow_(2).sum(1)

    @property
    def layout(self):
        return (torch.bfloat16, self.dp)

    def bind(self, x):
        # always re-derive the row norms: the caller may have refilled the same buffer
        if x.dtype != torch.bfloat16 or x.shape[1] != self.dp:
            raise ValueError(f"chunk layout {(x.dtype, x.shape[1])} != {self.layout}")
        self._set_x(x)
        return self

    def prepare(self, C):
        self.ops.finalize(None, None, C, 0, None, self.cm2, self.cnorm)

    def assign(self, C, labels, mind):
        self.ops.assign_bigd(self.x, None, self.xnorm, self.cm2, None, self.cnorm,
                             self._kg_for(self.x.shape[0]),
                             labels, mind, self._keys_for(self.n))

    def step(self, C, labels, mind, sums, counts):
        self.assign(C, labels, mind)
        self.update(self.x, labels, sums, counts)

    def finalize(self, sums, counts, C, shift):
        self.ops.finalize(sums, counts, C, self.policy, shift, self.cm2, self.cnorm,
                          fixed_scale=self.fixed_scale)

    def bf16_operands(self):
        return self.cm2, self.cnorm

    row_align = 32

    def pad_rows(self, kpad):
        if kpad != self.kp:
            self.kp = kpad
            self.cm2 = torch.zeros(kpad, self.dp, dtype=torch.bfloat16, device=self.device)
            self.cnorm = torch.zeros(kpad, dtype=torch.float32, device=self.device)
            self.kg = kgroup_tiles(self._row_bytes, self.kp, group_bytes=self.kgroup_bytes)

    def gather_operands(self):
        return [self.cm2, self.cnorm]

    def finalize_rows(self, sums, counts, C, shift, r0, kr):
        self.ops.finalize(sums, counts, C, self.policy, shift, self.cm2[r0:r0 + kr],
                          self.cnorm[r0:r0 + kr], fixed_scale=self.fixed_scale)

    def prep_rows(self, C, r0, kr):
        self.ops.finalize(None, None, C, 0, None, self.cm2[r0:r0 + kr], self.cnorm[r0:r0 + kr])


class HipFp8Lloyd(_GroupedAssign, _LocalOpsBase):
    """fp8 assignment (BASELINE config 5): the shard is quantised once to OCP e4m3 with
    one E8M0 exponent per 32 features (N8, `quant_fp8`); centroids are re-quantised each
    iteration as the -2c operand.  Distances run on the block-scaled MFMA; the update
    sums the full-precision shard (bf16/fp32), so centroids are exact means of the
    assigned points and fp8 only affects which centroid wins a near-tie."""
    name = "hip_fp8_mfma"
    c_dtype = torch.float32

    def __init__(self, x, k, empty_cluster="keep"):
        super().__init__(x, k, empty_cluster)
        self.ops = _native.require()
        self.dp = fp8_dim(self.d)
        if self.dp is None:
            raise ValueError(f"fp8 path supports D <= {FP8_DIMS[-1]}, got {self.d}")
        self.kp = ((k + 31) // 32) * 32
        dev = x.device
        self.cm2 = torch.zeros(self.kp, self.dp, dtype=torch.float8_e4m3fn, device=dev)
        self.cs = torch.zeros(self.kp, self.dp // 32, dtype=torch.uint8, device=dev)
        self.cnorm = torch.zeros(self.kp, dtype=torch.float32, device=dev)
        self._init_grouped(self.dp + self.dp // 32 + 4)
        self.x8 = self.xs = self.xnorm = None
        self.x = None
        self._set_x(x)
        self.update = NativeUpdate(self.ops, self.n, k, self.d, self.x.dtype, dev)

    def _set_x(self, x):
        if x.dtype == torch.float64:
            x = x.float()
        if not x.is_contiguous():
            x = x.contiguous()
        n = x.shape[0]
        if self.x8 is None or self.x8.shape[0] < n:
            self.x8 = torch.empty(n, self.dp, dtype=torch.float8_e4m3fn, device=x.device)
            self.xs = torch.empty(n, self.dp // 32, dtype=torch.uint8, device=x.device)
            self.xnorm = torch.empty(n, dtype=torch.float32, device=x.device)
        self.x = x
        self.n = n
        self.ops.quant_fp8(x[:, : self.d], n, 0, self.x8[:n], self.xs[:n], self.xnorm[:n])

    @property
    def layout(self):
        return (self.x.dtype, self.x.shape[1])

    def bind(self, x):
        # always re-quantise: the caller may have refilled the same buffer in place (a
        # serving layout buffer, a streaming ring slot), so identity says nothing
        if x.shape[1] != self.x.shape[1]:
            raise ValueError(f"chunk layout {(x.dtype, x.shape[1])} != {self.layout}")
        self._set_x(x)
        return self

    def prepare(self, C):
        self.ops.quant_fp8(C, self.k, 1, self.cm2, self.cs, self.cnorm)

    # near-tie re-check (ClusterConfig.fp8_recheck): where the fp8 margin between the
    # winner and the runner-up is within RECHECK_TAU of the runner-up's distance, both
    # distances are recomputed in fp32 from the full-precision rows.
    # Off by default: the top-2 epilogue costs ~8 % of the assignment (embed50m_fp8:
    # 1.93 -> 2.14 s/iter) for labels that only differ on near ties.  Needs one K-group
    # (N >= KGROUP_MIN_ITEMS * 256 rows per launch).  Set from ClusterConfig.fp8_recheck.
    RECHECK_TAU = 0.0

    def _top2_buffers(self, n):
        b = getattr(self, "_t2", None)
        if b is None or b[0].numel() < n:
            dev = self.device
            b = self._t2 = (torch.empty(n, dtype=torch.int32, device=dev),
                            torch.empty(n, dtype=torch.float32, device=dev),
                            torch.empty(n, dtype=torch.float32, device=dev))
        return b[0][:n], b[1][:n], b[2][:n]

    def assign(self, C, labels, mind):
        n = self.n
        kg = self._kg_for(n)
        if self.RECHECK_TAU > 0 and kg == 0:
            l2, d1, d2 = self._top2_buffers(n)
            self.ops.assign_bigd(self.x8[:n], self.xs[:n], self.xnorm[:n], self.cm2, self.cs,
                                 self.cnorm, 0, labels, d1, None, l2, d2)
            self.ops.recheck_top2(self.x, C.float().contiguous(), labels, l2, d1, d2,
                                  self.RECHECK_TAU)
        else:
            self.ops.assign_bigd(self.x8[:n], self.xs[:n], self.xnorm[:n], self.cm2, self.cs,
                                 self.cnorm, kg, labels, None, self._keys_for(n))
        if mind is not None:
            # inertia from the full-precision shard (the fp8 distances include the
            # quantisation noise of both operands; they only pick the winner)
            Cf = C.float()
            step = max(1, (1 << 28) // max(1, 4 * self.d))
            for s in range(0, n, step):
                e = min(n, s + step)
                diff = self.x[s:e, : self.d].float() - Cf.index_select(0, labels[s:e].long())
                mind[s:e] = diff.pow_(2).sum(1).to(mind.dtype)

    def step(self, C, labels, mind, sums, counts):
        self.assign(C, labels, mind)
        self.update(self.x, labels, sums, counts)

    def finalize(self, sums, counts, C, shift):
        self.ops.finalize(sums, counts, C, self.policy, shift, None, None,
                          fixed_scale=self.fixed_scale)
        self.prepare(C)

    def after_finalize(self, C):
        self.prepare(C)

    row_align = 32

    def pad_rows(self, kpad):
        if kpad != self.kp:
            dev = self.device
            self.kp = kpad
            self.cm2 = torch.zeros(kpad, self.dp, dtype=torch.float8_e4m3fn, device=dev)
            self.cs = torch.zeros(kpad, self.dp // 32, dtype=torch.uint8, device=dev)
            self.cnorm = torch.zeros(kpad, dtype=torch.float32, device=dev)
            self.kg = kgroup_tiles(self._row_bytes, self.kp, group_bytes=self.kgroup_bytes)

    def gather_operands(self):
        return [self.cm2, self.cs, self.cnorm]

    def finalize_rows(self, sums, counts, C, shift, r0, kr):
        # a rank whose rsag slice holds only padding rows (K small next to lcm(32, world))
        # finalises nothing but still writes its padding operands (quant of 0 rows: zeros
        # and the BIG pad norm)
        if C.shape[0]:
            self.ops.finalize(sums, counts, C, self.policy, shift, None, None,
                              fixed_scale=self.fixed_scale)
        self.prep_rows(C, r0, kr)

    def prep_rows(self, C, r0, kr):
        self.ops.quant_fp8(C, C.shape[0], 1, self.cm2[r0:r0 + kr], self.cs[r0:r0 + kr],
                           self.cnorm[r0:r0 + kr])


class _HipExactBase(_LocalOpsBase):
    def __init__(self, x, k, dtype, empty_cluster):
        super().__init__(x, k, empty_cluster)
        self.ops = _native.require()
        tdt = TORCH_DTYPES[dtype]
        self.x = x.to(tdt).contiguous()
        self.c_dtype = tdt
        self.update = NativeUpdate(self.ops, self.n, k, self.d, tdt, x.device)

    def finalize(self, sums, counts, C, shift):
        self.ops.finalize(sums, counts, C, self.policy, shift, None, None,
                          fixed_scale=self.fixed_scale)

    def finalize_rows(self, sums, counts, C, shift, r0, kr):
        if C.shape[0]:
            self.ops.finalize(sums, counts, C, self.policy, shift, None, None,
                              fixed_scale=self.fixed_scale)


class HipSmallLloyd(_HipExactBase):
    name = "hip_small_fused"

    def __init__(self, x, k, dtype, empty_cluster):
        super().__init__(x, k, dtype, empty_cluster)
        self.skip_step_labels = False  # set by the engine when a final label pass follows

    def supports_count_split(self) -> bool:
        return False  # the fused kernel accumulates counts itself (fp64 buffers only)

    def make_delta(self, *a, **kw):
        return None  # one fused assign + accumulate pass reads X once either way

    def step(self, C, labels, mind, sums, counts):
        self.ops.lloyd_small(self.x, C, None if self.skip_step_labels else labels, mind, sums,
                             counts)

    def assign(self, C, labels, mind):
        self.ops.assign_simt(self.x, C, labels, mind)


class HipSimtLloyd(_HipExactBase):
    name = "hip_simt"

    def step(self, C, labels, mind, sums, counts):
        self.ops.assign_simt(self.x, C, labels, mind)
        self.update(self.x, labels, sums, counts)

    def assign(self, C, labels, mind):
        self.ops.assign_simt(self.x, C, labels, mind)


class HipExactLloyd(_HipExactBase):
    """Large-D fp32/fp64: native tiled difference-form assignment (csrc/lloyd_simt.hip
    assign_exact, any D) + native update."""
    name = "hip_exact_tiled"

    def step(self, C, labels, mind, sums, counts):
        self.assign(C, labels, mind)
        self.update(self.x, labels, sums, counts)

    def assign(self, C, labels, mind):
        self.ops.assign_exact(self.x, C, labels, mind)


X3_DIMS = (32, 64, 128, 256)
X3_WIDE_MAX_D = 1024
X3_MIN_D = 16  # D <= 16: the SIMT / fused kernels (a 32-wide k-step would be mostly padding)


def x3_dim(d: int) -> Optional[int]:
    """Padded width of the fp32/fp64 MFMA assignment: 32/64/128/256 (register-resident
    point fragments), multiples of 128 up to 1024 (the row-chunk GEMM path), else None."""
    for p in X3_DIMS:
        if d <= p:
            return p
    if d <= X3_WIDE_MAX_D:
        return -(-d // 128) * 128
    return None


def _exact_mind(x: torch.Tensor, C: torch.Tensor, labels: torch.Tensor, mind: torch.Tensor, d: int):
    """mind[i] = ||x_i - C[labels_i]||^2 in the data's precision (inertia only: the MFMA
    scores pick the winner, the difference form gives the distance)."""
    n = x.shape[0]
    Cx = C.to(x.dtype)
    step = max(1, (1 << 28) // max(1, 8 * d))
    for s in range(0, n, step):
        e = min(n, s + step)
        diff = x[s:e, :d] - Cx.index_select(0, labels[s:e].long())
        mind[s:e] = diff.pow_(2).sum(1).to(mind.dtype)


class HipX3Lloyd(_LocalOpsBase):
    """fp32 / fp64 Lloyd with the assignment on the bf16 matrix cores (csrc/assign_x3.hip):
    rows and centroids split into bf16 hi/lo terms, scores from three MFMAs per product
    (fp32-faithful), the three smallest kept per row, and every row whose winner the
    error bound cannot certify re-checked exactly in the data's own dtype (the two
    candidates, or all K when a third is within the bound).  So the labels are those of
    the exact difference-form argmin (the reference's fp64 distances,
    `scripts/distribuitedClustering.py:221-234`), at ~1/3 of the bf16 MFMA rate instead of
    the vector rate.  D <= 256 keeps the point fragments in registers (the ring3
    pipeline); 256 < D <= 1024 runs the bf16x3 distance GEMM into a row-chunk block and a
    top-3 row pass.  The update, the all-reduce and the finalize use the fp32 / fp64 rows
    (NativeUpdate), as on the exact path.

    ``prefilter`` (D 33..256): a one-product pass first (xh . th, the bf16 ring3 kernel with
    top-2 and its own per-row bound, assign_mfma_impl.h x1_eps) labels every row whose gap
    certifies its winner and lists the rest; the three products then run over the listed
    rows only.  On clustered data most rows certify, so the step costs ~1/3 + the listed
    share of the full x3 pass; on data where nothing certifies it would cost ~4/3, so the
    listed count comes back to the host asynchronously (pinned copy + event, read when it
    has landed, never waited on) and a listed share above ``PRE_MAX_FRAC`` turns the
    prefilter off for ``PRE_RETRY`` assignments."""
    name = "hip_x3_mfma"
    chunk_elems = 1 << 27           # wide path: [rows, K] fp32 block per chunk
    max_chunk_rows = 1 << 20
    prefilter = True
    listed_estimate = True  # size the listed launch from the last listed share (A/B knob)
    PRE_MAX_FRAC = 0.6   # listed share above which the one-product pass costs more than it saves
    PRE_RETRY = 16

    def __init__(self, x, k, dtype="fp32", empty_cluster="keep"):
        super().__init__(x, k, empty_cluster)
        self.ops = _native.require()
        self.c_dtype = TORCH_DTYPES[dtype]
        self.dp = x3_dim(self.d)
        if self.dp is None or dtype not in ("fp32", "fp64"):
            raise ValueError(f"x3 path: fp32/fp64 with D <= {X3_WIDE_MAX_D}, got {dtype} D={self.d}")
        self.wide = self.dp > X3_DIMS[-1]
        self.kp = -(-k // (128 if self.wide else 64)) * (128 if self.wide else 64)
        dev = x.device
        self.ch = torch.zeros(self.kp, self.dp, dtype=torch.bfloat16, device=dev)
        self.cl = torch.zeros_like(self.ch)
        self.cnorm = torch.zeros(self.kp, dtype=torch.float32, device=dev)
        self.cnhl = torch.zeros(self.kp, 2, dtype=torch.float32, device=dev)  # ||th||^2, ||tl||^2
        self.cstat = torch.zeros(3, dtype=torch.float32, device=dev)  # maxima of cnorm / cnhl
        # [0] two-candidate list, [1] full re-scan list, [2] the prefilter's listed rows
        self.amb_count = torch.zeros(3, dtype=torch.int32, device=dev)
        self.xh = self.xl = self.xx = self.amb = self.G = self.pre = self.xnhl = None
        self.x = self.mu = None
        self._set_x(x)
        self.update = NativeUpdate(self.ops, self.n, k, self.d, self.c_dtype, dev)

    def _set_x(self, x):
        if x.dtype != self.c_dtype or x.stride(-1) != 1:
            x = x.to(self.c_dtype).contiguous()
        n = int(x.shape[0])
        if self.xh is None or self.xh.shape[0] < n:
            dev = self.device
            self.xh = torch.empty(max(n, 1), self.dp, dtype=torch.bfloat16, device=dev)
            self.xl = torch.empty_like(self.xh)
            self.xx = torch.empty(max(n, 1), dtype=torch.float32, device=dev) if self.wide else None
            # re-check lists: int2 {row, runner-up} entries | full re-scan rows
            self.amb = torch.empty(3 * max(n, 1), dtype=torch.int32, device=dev)
            pre_ok = self.dp in (64, 128, 256)
            self.pre = torch.empty(max(n, 1), dtype=torch.int32, device=dev) if pre_ok else None
            # ||xh||^2, ||xl||^2 per row: the prefilter's bound takes the row's own residual
            self.xnhl = torch.empty(max(n, 1), 2, dtype=torch.float32, device=dev) if pre_ok else None
        self.x = x
        self.n = n
        if self.mu is None and n >= 2:
            # fixed shift (this rank's first rows' mean; a streamed engine's one-row probe:
            # the first centroids' mean, set in prepare): rows and centroids are split as
            # v - mu, so the error bounds scale with the data's spread, not its offset
            # (uncentred data otherwise fails the bound and re-scans exactly); the argmin
            # is shift-invariant and the exact re-check reads the unshifted rows
            self.mu = x[:, : self.d].double().mean(0).to(self.c_dtype).contiguous()
        self._split_rows()

    def _split_rows(self):
        n, x = self.n, self.x
        if n:
            self.ops.x3_split(x[:, : self.d], n, 0, self.xh[:n], self.xl[:n],
                              self.xx[:n] if self.wide else None,
                              self.xnhl[:n] if self.xnhl is not None else None, self.mu)

    @property
    def layout(self):
        return (self.c_dtype, self.d)

    def bind(self, x):
        # always re-split: a streaming slot is refilled in place
        if x.shape[1] != self.d:
            raise ValueError(f"chunk layout {(x.dtype, x.shape[1])} != {self.layout}")
        self._set_x(x)
        return self

    def prepare(self, C):
        Cx = C.to(self.c_dtype).contiguous()
        if self.mu is None:
            self.mu = Cx[: self.k, : self.d].double().mean(0).to(self.c_dtype).contiguous()
            self._split_rows()  # rows already split without it
        self.ops.x3_split(Cx, self.k, 1, self.ch, self.cl, self.cnorm, self.cnhl, self.mu)

    def _chunk_rows(self):
        rows = max(1, min(self.n, self.chunk_elems // max(1, self.k), self.max_chunk_rows))
        if self.G is None or self.G.shape[0] < rows:
            self.G = torch.empty(rows, self.k, dtype=torch.float32, device=self.device)
        return rows

    def assign(self, C, labels, mind):
        n = self.n
        if n == 0:
            return
        Cx = C if (C.dtype == self.c_dtype and C.is_contiguous()) else C.to(self.c_dtype).contiguous()
        amb = self.amb[: 3 * n]  # the lists' layout follows their capacity: n rows
        if not self.wide:
            pre = self.pre if self._want_prefilter() else None
            self._pre_ran = pre is not None
            # the listed launch is sized from the last listed share that came back (+25 %
            # and a margin; anything beyond goes to a small grid-stride launch)
            frac = getattr(self, "_pre_frac", None) if self.listed_estimate else None
            est = -1 if frac is None else min(n, int(frac * n * 1.25) + 16384)
            self.ops.x3_assign(self.x, self.xh[:n], self.xl[:n], self.ch, self.cl, self.cnorm,
                               self.cnhl, Cx, labels, None, amb, self.cstat, self.amb_count, True,
                               pre, self.xnhl[:n] if pre is not None else None, est)
            if pre is not None and self._pre_ev is None and \
                    not torch.cuda.is_current_stream_capturing():
                # the count goes to the host on a side stream (a D2H blit on the compute
                # stream held it ~38 us per step, profiles/fp64_2m_ksplit_kernel_stats_r06h.txt),
                # from a device snapshot that is rewritten only after this copy has landed
                if getattr(self, "_copy_stream", None) is None:
                    self._copy_stream = torch.cuda.Stream(device=self.device)
                    self._pre_snap = torch.zeros(1, dtype=torch.int32, device=self.device)
                self._pre_snap.copy_(self.amb_count[2:3])
                ev0 = torch.cuda.Event()
                ev0.record()
                self._copy_stream.wait_event(ev0)
                with torch.cuda.stream(self._copy_stream):
                    self._pre_host.copy_(self._pre_snap, non_blocking=True)
                    self._pre_ev = torch.cuda.Event()
                    self._pre_ev.record(self._copy_stream)
                self._pre_n = n
        else:
            self.ops.x3_prep(self.cnorm, self.cnhl, self.k, self.cstat, self.amb_count)
            rows = self._chunk_rows()
            for s in range(0, n, rows):
                e = min(n, s + rows)
                g = self.G[: e - s]
                self.ops.fcm_mfma_wide(1, self.xh[s:e], self.xl[s:e], self.xx[s:e], self.ch,
                                       self.cl, self.cnorm, self.k, self.d, g)
                self.ops.x3_rows(g, s, self.xx[s:e], self.cstat, self.dp, labels, amb,
                                 self.amb_count)
            self.ops.x3_recheck(self.x, Cx, labels, amb, self.amb_count)
        if mind is not None:
            _exact_mind(self.x, C, labels, mind, self.d)

    def _want_prefilter(self) -> bool:
        if not self.prefilter or self.pre is None:
            return False
        if not hasattr(self, "_pre_ev"):
            self._pre_ev, self._pre_off, self._pre_n = None, 0, 0
            self._pre_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        if torch.cuda.is_current_stream_capturing():
            return self._pre_off == 0  # a captured step keeps the current choice
        if self._pre_off > 0:
            self._pre_off -= 1
            return False
        ev = self._pre_ev
        if ev is not None and ev.query():  # the count of an earlier assignment has landed
            self._pre_ev = None
            self._pre_frac = int(self._pre_host[0]) / max(1, self._pre_n)
            if int(self._pre_host[0]) > self.PRE_MAX_FRAC * max(1, self._pre_n):
                self._pre_off = self.PRE_RETRY - 1
                return False
        return True

    def settle(self):
        """Wait for the last assignment's listed count and take it in (before a graph
        capture: the replay keeps the prefilter choice and sizes the listed launch from
        this share, instead of the full-size launch of an unknown share)."""
        ev = getattr(self, "_pre_ev", None)
        if ev is not None:
            ev.synchronize()
            self._want_prefilter()

    def ambiguous_rows(self) -> int:
        """Rows the last assignment re-checked exactly (host read; diagnostics)."""
        return int(self.amb_count[:2].sum().item())

    def prefilter_rows(self) -> int:
        """Rows the last assignment's one-product prefilter left to the three-product pass
        (0 when the prefilter did not run; host read; diagnostics)."""
        return int(self.amb_count[2].item()) if getattr(self, "_pre_ran", False) else 0

    def rescanned_rows(self) -> int:
        """... of which re-scanned over all K (a third candidate within the bound)."""
        return int(self.amb_count[1].item())

    def step(self, C, labels, mind, sums, counts):
        self.assign(C, labels, mind)
        self.update(self.x, labels, sums, counts)

    def finalize(self, sums, counts, C, shift):
        self.ops.finalize(sums, counts, C, self.policy, shift, None, None,
                          fixed_scale=self.fixed_scale)
        self.prepare(C)

    def after_finalize(self, C):
        self.prepare(C)

    def after_gather(self, C):
        self.prepare(C)

    def finalize_rows(self, sums, counts, C, shift, r0, kr):
        # rsag: the exact centroid rows are what the ranks all-gather (the re-check reads
        # them; as many bytes as the hi/lo images), the operands are prepped after it
        if C.shape[0]:
            self.ops.finalize(sums, counts, C, self.policy, shift, None, None,
                              fixed_scale=self.fixed_scale)


def lloyd_row_extra(dtype: str, d: int, delta: bool = True) -> int:
    """Device bytes per row a Lloyd shard holds besides its layout row (the HBM planner's
    per_row_extra): labels + min distances + the sorted update's permutation (16), the delta
    update's prev / moved-list / event permutation (20), and on the fp32 / fp64 MFMA path
    the bf16 hi/lo rows (4 x padded D) + the re-check list entries (12) + the prefilter's
    list entry and the row's split norms (12)."""
    extra = 16 + (20 if delta else 0)
    if dtype in ("fp32", "fp64") and d > X3_MIN_D and x3_dim(d) is not None:
        extra += 4 * x3_dim(d) + 24
    return extra


def lloyd_fixed_extra(k: int, d: int, delta: bool = True, dtype: Optional[str] = None,
                      n: Optional[int] = None) -> int:
    """Device bytes a Lloyd shard holds independent of its rows beyond the planner's
    default: the delta update's fp64 running totals; on the wide fp32 / fp64 MFMA path
    (HipX3Lloyd, D > 256) the [rows, K] fp32 score block of a row chunk; and the
    inertia pass's difference block (_exact_mind, 2^28 bytes)."""
    extra = (k * d + k) * 8 if delta else 0
    if dtype in ("fp32", "fp64") and d > X3_MIN_D and x3_dim(d) is not None:
        if x3_dim(d) > X3_DIMS[-1]:
            rows = min(n if n is not None else HipX3Lloyd.max_chunk_rows,
                       HipX3Lloyd.chunk_elems // max(1, k), HipX3Lloyd.max_chunk_rows)
            extra += max(1, rows) * k * 4
        extra += 1 << 28
    return extra


def lloyd_layout(dtype: str, d: int):
    """(torch dtype, width) of the rows the GPU Lloyd ops for ``dtype`` consume (the
    layout a streamed source must produce; mirrors :func:`_make_lloyd_ops`)."""
    if dtype == "fp8" and fp8_dim(d) is not None:
        return (torch.float32, d)  # fp8 ops quantise each chunk they are bound to
    if dtype in ("bf16", "fp8"):
        w = padded_dim(d) or wide_bf16_dim(d)
        return (torch.bfloat16, w) if w is not None else (torch.float32, d)
    return (TORCH_DTYPES[dtype], d)


def make_lloyd_ops(x: torch.Tensor, k: int, dtype: str = "bf16", backend: str = "auto",
                   empty_cluster: str = "keep", deterministic: bool = False,
                   kgroup_bytes: int = 0, fp8_recheck: float = 0.0, exact_assign: str = "auto"):
    """Pick the fastest local implementation for (device, dtype, K, D).

    ``kgroup_bytes`` / ``fp8_recheck``: ClusterConfig tunables of the wide-D / fp8 assign
    (K-group size; near-tie re-check margin), applied to the ops that have them.
    ``exact_assign`` (fp32 / fp64): 'auto' / 'mfma' = the bf16x3 MFMA assignment with the
    exact re-check (HipX3Lloyd) for 16 < D <= 1024; 'simt' = the difference-form SIMT
    tiles (the same labels up to the dtype's rounding, at the vector rate)."""
    ops = _make_lloyd_ops(x, k, dtype, backend, empty_cluster, deterministic, exact_assign)
    upd = getattr(ops, "update", None)
    if deterministic and isinstance(upd, NativeUpdate) and not upd.deterministic:
        # fixed-point partials: always the sorted path (the LDS path sums in float atomics)
        ops.update = NativeUpdate(upd.ops, ops.n, k, ops.d, ops.x.dtype, ops.device,
                                  deterministic=True)
    if isinstance(ops, _GroupedAssign) and kgroup_bytes:
        ops.kgroup_bytes = int(kgroup_bytes)
        ops.kg = kgroup_tiles(ops._row_bytes, ops.kp, group_bytes=ops.kgroup_bytes)
    if isinstance(ops, HipFp8Lloyd) and fp8_recheck > 0:
        ops.RECHECK_TAU = float(fp8_recheck)
    return ops


def _make_lloyd_ops(x, k, dtype, backend, empty_cluster, deterministic, exact_assign="auto"):
    d = x.shape[1]
    if not use_native(x.device, backend):
        return TorchLloyd(x, k, dtype if dtype in ("fp64", "fp32") else "fp32", empty_cluster)
    if dtype == "fp8":
        if fp8_dim(d) is not None:
            return HipFp8Lloyd(x, k, empty_cluster)
        dtype = "bf16"  # D > 1024: bf16/fp32 paths below
    if dtype == "bf16":
        if padded_dim(d) is not None:
            return HipBf16Lloyd(x, k, empty_cluster)
        if wide_bf16_dim(d) is not None:
            return HipWideBf16Lloyd(x, k, empty_cluster)
        return HipExactLloyd(x, k, "fp32", empty_cluster)  # bf16 D > 1024: exact fp32 tiles
    tdt = TORCH_DTYPES[dtype]
    ops = _native.require()
    if ops.lloyd_small_supported(tdt, k, d) and not deterministic:
        return HipSmallLloyd(x, k, dtype, empty_cluster)
    if exact_assign != "simt" and d > X3_MIN_D and x3_dim(d) is not None:
        return HipX3Lloyd(x, k, dtype, empty_cluster)
    if d <= (64 if dtype == "fp32" else 32):
        return HipSimtLloyd(x, k, dtype, empty_cluster)
    return HipExactLloyd(x, k, dtype, empty_cluster)


# ----------------------------------------------------------------------------- FCM
class TorchFCM(_LocalOpsBase):
    name = "torch_fcm"

    def __init__(self, x, k, dtype="fp64", m=2.0, nan_to_zero=True):
        super().__init__(x, k, "keep")
        tdt = torch.float64 if dtype == "fp64" else torch.float32
        self.x = x.to(tdt).contiguous()
        self.c_dtype = tdt
        self.m = float(m)
        self.nan_to_zero = nan_to_zero

    def step(self, C, labels, wx, ws):
        a, b, lab = ref.fcm_partial(self.x, C.to(self.x.dtype), self.m, self.nan_to_zero,
                                    acc_dtype=wx.dtype)
        wx.add_(a)
        ws.add_(b)
        labels.copy_(lab)

    def assign(self, C, labels):
        c = C.to(self.x.dtype)
        step = max(1, (1 << 26) // max(1, self.k))  # bound the [rows, K] membership block
        for s in range(0, self.n, step):
            u = ref.fcm_memberships(self.x[s:s + step], c, self.m, self.nan_to_zero)
            labels[s:s + step] = u.argmax(1).to(torch.int32)


class HipSmallFCM(_LocalOpsBase):
    name = "hip_fcm_small"

    def __init__(self, x, k, dtype="fp64", m=2.0, nan_to_zero=True):
        super().__init__(x, k, "keep")
        self.ops = _native.require()
        tdt = torch.float64 if dtype == "fp64" else torch.float32
        self.x = x.to(tdt).contiguous()
        self.c_dtype = tdt
        self.m = float(m)
        self.nan_to_zero = nan_to_zero
        self._wx = None
        self.skip_step_labels = False  # set by the engine when a final label pass follows

    def step(self, C, labels, wx, ws):
        self.ops.fcm_small(self.x, C, self.m, self.nan_to_zero,
                           None if self.skip_step_labels else labels, wx, ws)

    def assign(self, C, labels):
        if self._wx is None:
            self._wx = torch.zeros(self.k, self.d, dtype=torch.float64, device=self.device)
            self._ws = torch.zeros(self.k, dtype=torch.float64, device=self.device)
        self.ops.fcm_small(self.x, C, self.m, self.nan_to_zero, labels, self._wx, self._ws)

    def finalize(self, sums, counts, C, shift):
        self.ops.finalize(sums, counts, C, 0, shift, None, None)


class HipTowerFCM(_LocalOpsBase):
    """FCM for any K and D <= 256 in fp32 / fp64 (csrc/fcm_tower.hip): a stats pass (row
    normaliser + argmax label per row, exact difference-form distances) and an accumulate
    pass (centroid tile x row range: the tile's sum_i w x_i and sum_i w in registers).
    No host syncs; ``rowinfo`` [N] is the only intermediate."""
    name = "hip_fcm_tower"

    def __init__(self, x, k, dtype="fp64", m=2.0, nan_to_zero=True):
        super().__init__(x, k, "keep")
        self.ops = _native.require()
        tdt = torch.float64 if dtype == "fp64" else torch.float32
        self.x = x.to(tdt).contiguous()
        self.c_dtype = tdt
        self.m = float(m)
        self.nan_to_zero = bool(nan_to_zero)
        self.rowinfo = torch.empty(self.n, dtype=tdt, device=self.device)
        self._wx = self._ws = None

    def bind(self, x):
        super().bind(x)
        if self.rowinfo.numel() < self.n:
            self.rowinfo = torch.empty(self.n, dtype=self.c_dtype, device=self.device)
        return self

    def step(self, C, labels, wx, ws):
        C = C.to(self.c_dtype).contiguous()
        ri = self.rowinfo[: self.n]
        self.ops.fcm_tower_stats(self.x, C, self.m, self.nan_to_zero, labels, ri)
        self.ops.fcm_tower_accum(self.x, C, self.m, self.nan_to_zero, ri, wx, ws)

    def assign(self, C, labels):
        self.ops.fcm_tower_stats(self.x, C.to(self.c_dtype).contiguous(), self.m,
                                 self.nan_to_zero, labels, self.rowinfo[: self.n])

    def finalize(self, sums, counts, C, shift):
        self.ops.finalize(sums, counts, C, 0, shift, None, None)


FCM_MFMA_DIMS = (32, 64, 128)
FCM_MFMA_MIN_K = 32  # below: the SIMT tower (a 128-centroid MFMA tile would be mostly padding)


def fcm_mfma_dim(d: int) -> Optional[int]:
    for p in FCM_MFMA_DIMS:
        if d <= p:
            return p
    return None


class HipMfmaFCM(_LocalOpsBase):
    """bf16 / fp8 FCM (``--dtype bf16``) on bf16 matrix cores (csrc/fcm_mfma.hip); fp32 and
    fp64 FCM run the exact towers instead (make_fcm_ops).  The shard is split once into
    hi/lo bf16 rows (+ fp32 norms), the centroids every iteration; a stats pass (row
    normaliser + label) and an accumulate pass (distances -> w -> W^T X, all on MFMA)."""
    name = "hip_fcm_mfma"

    @staticmethod
    def _pick_dp(d: int) -> Optional[int]:
        return fcm_mfma_dim(d)

    def __init__(self, x, k, m=2.0, nan_to_zero=True):
        super().__init__(x, k, "keep")
        self.ops = _native.require()
        self.dp = self._pick_dp(self.d)
        if self.dp is None:
            raise ValueError(f"{type(self).__name__} does not support D = {self.d}")
        self.c_dtype = torch.float32
        self.m = float(m)
        self.nan_to_zero = bool(nan_to_zero)
        self.kp = -(-k // 128) * 128
        dev = self.device
        self.ch = torch.zeros(self.kp, self.dp, dtype=torch.bfloat16, device=dev)
        self.cl = torch.zeros_like(self.ch)
        self.cc = torch.zeros(self.kp, dtype=torch.float32, device=dev)
        self.xh = self.xl = self.xx = self.rowinfo = self.xr = None
        self.work = self.mu = None
        self._set_x(x)

    @property
    def layout(self):
        return (torch.float32, self.d)

    def _work(self):
        need = int(self.ops.fcm_mfma_workspace(self.cc, self.n, self.k, self.kp, self.dp))
        if self.work is None or self.work.numel() < need:
            self.work = torch.empty(need, dtype=torch.float32, device=self.device)
        return self.work

    def _set_x(self, x, streamed: bool = False):
        """Hold the rows; they are split into hi/lo at the next step, once the shift (the
        mean of the first centroids -- replicated, so resident, streamed and every world
        size use the same one) is known."""
        self._xsrc = x if (x.dtype == torch.float32 and x.stride(1) == 1) else x.float().contiguous()
        # bf16 rows are also the exact W^T X operand of the one-product accumulate (Xr);
        # a streamed chunk is copied (its buffer is refilled while the step may still read)
        self._xraw = x if x.dtype == torch.bfloat16 else None
        self._xraw_alias = not streamed
        self.n = int(x.shape[0])
        self._dirty = True
        self.x = None

    def _split_x(self):
        n = self.n
        if self.xh is None or self.xh.shape[0] < n:
            dev = self.device
            self.xh = torch.empty(n, self.dp, dtype=torch.bfloat16, device=dev)
            self.xl = torch.empty_like(self.xh)
            self.xx = torch.empty(n, dtype=torch.float32, device=dev)
            self.rowinfo = None
        # row statistics + (DP >= 64) the two corrected nearest d2 per row, which let the
        # accumulate pass run one-product distances
        ril = self._ri_len(n)
        if self.rowinfo is None or self.rowinfo.numel() < ril:
            self.rowinfo = torch.empty(ril, dtype=torch.float32, device=self.device)
        self.ops.fcm_split_rows(self._xsrc[:, : self.d], n, 0, self.xh[:n], self.xl[:n],
                                self.xx[:n], self.mu)
        self._xsrc = None  # the hi/lo rows are the shard from here on
        self.xr = None
        if self._xraw is not None and self._use_raw():
            xr = self._xraw[:, : self.d]
            if self.d == self.dp and xr.is_contiguous() and self._xraw_alias:
                self.xr = xr  # the shard itself
            else:
                # an owned, zero-padded copy (reused by the next streamed chunk)
                buf = getattr(self, "_xr_buf", None)
                if buf is None or buf.shape[0] < n:
                    buf = self._xr_buf = torch.zeros(n, self.dp, dtype=torch.bfloat16,
                                                     device=self.device)
                self.xr = buf[:n]
                self.xr[:, : self.d] = xr
        self._xraw = None
        self._dirty = False

    def bind(self, x):
        if x.shape[1] != self.d:
            raise ValueError(f"chunk width {x.shape[1]} != {self.d}")
        self._set_x(x, streamed=True)
        return self

    def prepare(self, C):
        Cf = C.float().contiguous()
        if self.mu is None:
            # fixed shift: distances are shift-invariant and the expansion's cancellation
            # error scales with |x - mu|^2 instead of |x|^2
            self.mu = Cf.double().mean(0).float()
        self.ops.fcm_split_rows(Cf, self.k, 1, self.ch, self.cl, self.cc, self.mu)
        if self._dirty:
            self._split_x()

    def _ops_args(self):
        n = self.n
        return self.xh[:n], self.xl[:n], self.xx[:n]

    # one-product accumulate (ClusterConfig.fcm_distances = 'one'); off: bf16x3 distances
    one_product = False
    raw_rows = True     # class switch: bf16 shards feed W^T X as they are (one product)

    def _use_raw(self):
        return self.raw_rows and self.dp >= 64

    @property
    def precision(self) -> str:
        """What the step computes, in words (bench.py reports it)."""
        raw = getattr(self, "xr", None) is not None
        if self.one_product and self.dp >= 64:
            return FCM_PRECISION["bf16_one_raw" if raw else "bf16_one"]
        return FCM_PRECISION["bf16_raw" if raw else "bf16"]

    def _ri_len(self, n):
        if not self.one_product:
            return n
        return int(self.ops.fcm_mfma_rowinfo_len(self.cc, n, self.dp))

    def step(self, C, labels, wx, ws):
        self.prepare(C)
        xh, xl, xx = self._ops_args()
        ri = self.rowinfo[: self._ri_len(self.n)]
        self.ops.fcm_mfma_stats(xh, xl, xx, self.ch, self.cl, self.cc, self.k, self.m,
                                self.nan_to_zero, labels, ri)
        xr = self.xr[: self.n] if self.xr is not None else None
        self.ops.fcm_mfma_accum(xh, xl, xx, ri, self.ch, self.cl, self.cc, self.k, self.m,
                                self.nan_to_zero, wx, ws, self._work(), self.mu, xr)

    def assign(self, C, labels):
        self.prepare(C)
        xh, xl, xx = self._ops_args()
        self.ops.fcm_mfma_stats(xh, xl, xx, self.ch, self.cl, self.cc, self.k, self.m,
                                self.nan_to_zero, labels, self.rowinfo[: self.n])

    def finalize(self, sums, counts, C, shift):
        self.ops.finalize(sums, counts, C, 0, shift, None, None)


FCM_MFMA_WIDE_MAX_D = 1024


def fcm_mfma_wide_dim(d: int) -> Optional[int]:
    """Padded width (a multiple of 128) of the wide MFMA FCM path, 128 < D <= 1024."""
    if d <= FCM_MFMA_DIMS[-1] or d > FCM_MFMA_WIDE_MAX_D:
        return None
    return -(-d // 128) * 128


class HipMfmaWideFCM(HipMfmaFCM):
    """bf16 / fp8 FCM for 128 < D <= 1024 on bf16 matrix cores (csrc/fcm_mfma.hip wide_*): the
    tower's hi/lo operands no longer fit a wave's registers, so each row chunk runs
    three native kernels with its [rows, K] block G in HBM, like HipWideFCM, but with both
    products on MFMA: distances (xh ch + xh cl + xl ch) into G, memberships w = u^m in
    place (the wide tower's row pass), then W^T X from G and the hi/lo rows (W split into
    hi/lo bf16 on its way through LDS) into per-split slabs reduced in fp64."""
    name = "hip_fcm_mfma"
    chunk_elems = 1 << 27
    max_chunk_rows = 1 << 20  # keeps every per-split X offset of the W^T X pass in 32 bits

    one_product = False  # no stats-pass fix-up rows on the wide path

    @staticmethod
    def _pick_dp(d: int) -> Optional[int]:
        return fcm_mfma_wide_dim(d)

    def __init__(self, x, k, m=2.0, nan_to_zero=True):
        self.G = None
        self._wwork = None
        super().__init__(x, k, m, nan_to_zero)

    def _block(self):
        rows = max(1, min(self.n, self.chunk_elems // max(1, self.k), self.max_chunk_rows))
        if self.G is None or self.G.shape[0] < rows:
            self.G = torch.empty(rows, self.k, dtype=torch.float32, device=self.device)
        need = int(self.ops.fcm_mfma_wide_workspace(self.cc, rows, self.kp, self.dp))
        if self._wwork is None or self._wwork.numel() < need:
            self._wwork = torch.empty(need, dtype=torch.float32, device=self.device)
        return rows

    def _chunks(self):
        rows = self._block()
        for s in range(0, self.n, rows):
            e = min(self.n, s + rows)
            yield s, e, self.G[: e - s]

    def step(self, C, labels, wx, ws):
        self.prepare(C)
        k, d = self.k, self.d
        for s, e, g in self._chunks():
            xh, xl, xx = self.xh[s:e], self.xl[s:e], self.xx[s:e]
            self.ops.fcm_mfma_wide(0, xh, xl, xx, self.ch, self.cl, self.cc, k, d, g)
            self.ops.fcm_wide_rows(g, k, self.m, self.nan_to_zero, labels[s:e], True)
            self.ops.fcm_mfma_wide(2, xh, xl, xx, self.ch, self.cl, self.cc, k, d, g,
                                   self._wwork, self.mu, wx, ws)

    def assign(self, C, labels):
        self.prepare(C)
        k, d = self.k, self.d
        for s, e, g in self._chunks():
            self.ops.fcm_mfma_wide(0, self.xh[s:e], self.xl[s:e], self.xx[s:e], self.ch, self.cl,
                                   self.cc, k, d, g)
            self.ops.fcm_wide_rows(g, k, self.m, self.nan_to_zero, labels[s:e], False)


class HipWideFCM(_LocalOpsBase):
    """FCM for any D in fp32 / fp64 (csrc/fcm_wide.hip) per row chunk, with the [rows, K]
    block G (up to ``chunk_elems`` elements) as the only intermediate, no library GEMM.

    fp64 (``fused``, the default): two kernels per chunk, both GEMM-shaped passes on the f64
    matrix cores -- the distance expansion with an exact-zero bound, t = d^(-2/(m-1)) into G
    and the row statistics (sum t, on-centroid count, label) in the same kernel, then
    W^T X with w = (t / sum t)^m formed while staging.  Unfused fp64 / fp32: distances
    into G, memberships w = u^m in place (fcm_wide_rows), W^T X -- three kernels per chunk
    (fp32 on exact difference-form SIMT tiles)."""
    name = "hip_fcm_wide"
    # [rows, K] block per chunk (2 GiB in fp64): each chunk's W^T X pass flushes its
    # partial tiles with atomics and ends in a partial round of blocks, so fewer, larger
    # chunks; HBM is 288 GB per GPU
    chunk_elems = 1 << 28
    fused = True  # class switch (A/B): fp64 row statistics fused into the distance pass

    def __init__(self, x, k, dtype="fp64", m=2.0, nan_to_zero=True):
        super().__init__(x, k, "keep")
        self.ops = _native.require()
        tdt = torch.float64 if dtype == "fp64" else torch.float32
        self.promoted = tdt == torch.float64 and x.dtype != torch.float64
        self.x = x.to(tdt).contiguous()
        self.c_dtype = tdt
        self.m = float(m)
        self.nan_to_zero = bool(nan_to_zero)
        self.G = None
        self.rowinfo = None

    @property
    def precision(self) -> str:
        if self._fused():
            return FCM_PRECISION["fp64_mfma"] + (" (fp32 rows promoted to fp64)"
                                                 if self.promoted else "")
        return FCM_PRECISION["fp64" if self.c_dtype == torch.float64 else "fp32"]

    def _fused(self) -> bool:
        return self.fused and self.c_dtype == torch.float64

    def bind(self, x):
        """A streamed chunk; fp32 chunks of a promoted shard are widened into an owned
        fp64 buffer (the source refills its slot while the step may still read)."""
        if x.shape[1] != self.d:
            raise ValueError(f"chunk width {x.shape[1]} != {self.d}")
        if x.dtype == self.c_dtype:
            self.x = x
        else:
            buf = getattr(self, "_xbuf", None)
            if buf is None or buf.shape[0] < x.shape[0]:
                buf = self._xbuf = torch.empty(x.shape[0], self.d, dtype=self.c_dtype,
                                               device=self.device)
            self.x = buf[: x.shape[0]]
            self.x.copy_(x)
        self.n = x.shape[0]
        return self

    def _block(self):
        rows = max(1, min(self.n, self.chunk_elems // max(1, self.k)))
        if self.G is None or self.G.shape[0] < rows:
            self.G = torch.empty(rows, self.k, dtype=self.c_dtype, device=self.device)
        if self._fused() and (self.rowinfo is None or self.rowinfo.numel() < rows):
            self.rowinfo = torch.empty(rows, dtype=torch.float64, device=self.device)
        return rows

    def _chunks(self):
        rows = self._block()
        for s in range(0, self.n, rows):
            e = min(self.n, s + rows)
            yield s, e, self.x[s:e], self.G[: e - s]

    def step(self, C, labels, wx, ws):
        C = C.to(self.c_dtype).contiguous()
        for s, e, xs, g in self._chunks():
            if self._fused():
                ri = self.rowinfo[: e - s]
                self.ops.fcm_f64t(0, xs, C, self.m, self.nan_to_zero, g, ri, labels[s:e])
                self.ops.fcm_f64t(1, xs, C, self.m, self.nan_to_zero, g, ri, None, wx, ws)
                continue
            self.ops.fcm_wide(0, xs, C, self.m, self.nan_to_zero, g)
            self.ops.fcm_wide(1, xs, C, self.m, self.nan_to_zero, g, labels[s:e])
            self.ops.fcm_wide(2, xs, C, self.m, self.nan_to_zero, g, None, wx, ws)

    def assign(self, C, labels):
        C = C.to(self.c_dtype).contiguous()
        for s, e, xs, g in self._chunks():
            if self._fused():
                self.ops.fcm_f64t(0, xs, C, self.m, self.nan_to_zero, g,
                                  self.rowinfo[: e - s], labels[s:e])
                continue
            self.ops.fcm_wide(0, xs, C, self.m, self.nan_to_zero, g)
            self.ops.fcm_wide(3, xs, C, self.m, self.nan_to_zero, g, labels[s:e])

    def finalize(self, sums, counts, C, shift):
        self.ops.finalize(sums, counts, C, 0, shift, None, None)


# what each FCM dtype computes (bench.py / --extended_log report it)
FCM_PRECISION = {
    "fp64": "fp64 distances (difference form; D > 256: the GEMM expansion on the fp64 matrix "
            "cores), fp64 memberships and sums",
    "fp32": "fp32 difference-form distances and memberships, fp64 sums",
    # HipWideFCM fused fp64 (also fp32 data promoted to it where make_fcm_ops routes so)
    "fp64_mfma": "fp64 distances as the GEMM expansion on the fp64 matrix cores (exact-zero "
                 "bound (3D+4) 2^-53 (|x|+|c|)^2), fp64 memberships, W^T X on the fp64 "
                 "matrix cores, fp64 sums",
    # HipMfmaFCM, fcm_distances='x3' (default): bf16x3 in both passes.  bf16 hi + lo hold 16
    # of fp32's 24 mantissa bits, so a product carries ~3 2^-16 |x||c| of error -- relative
    # to a small d2 next to a centroid that is percent-level on tight, well-separated
    # clusters (the fcm10m witness); sum w within ~2e-3*m of fp64 on the oracle tests
    "bf16": "bf16x3 MFMA distances in both passes (|d2 error| ~ 3 2^-16 |x-mu||c-mu|), "
            "fp32 memberships, bf16 weights in the W^T X MFMAs (hi+lo rows), fp64 sums",
    # ... on a bf16 shard from D = 64: W^T X takes the bf16 rows themselves (exact products)
    "bf16_raw": "bf16x3 MFMA distances in both passes (|d2 error| ~ 3 2^-16 "
                "|x-mu||c-mu|), fp32 memberships; W^T X = bf16 weights x the bf16 rows (exact "
                "products, fp32 accumulate), fp64 sums",
    # HipMfmaFCM from D = 64, fcm_distances='one': both passes one product + the fix-up
    "bf16_one": "both passes: one bf16 product (x_hi . c_hi, ~2^-9/sqrt(D) relative error "
                "on x.c) per centroid, each row's two nearest corrected to bf16x3; fp32 "
                "memberships, bf16 weights in the W^T X MFMAs (hi+lo rows), fp64 sums",
    # ... on a bf16 shard: W^T X takes the bf16 rows themselves (exact products)
    "bf16_one_raw": "both passes: one bf16 product (x_hi . c_hi, ~2^-9/sqrt(D) relative "
                    "error on x.c) per centroid, each row's two nearest corrected to bf16x3; "
                    "fp32 memberships; W^T X = bf16 weights x the bf16 rows (exact products, "
                    "fp32 accumulate), fp64 sums",
}


# A/B switch of make_fcm_ops (bench.py --fcm-path): "" = the measured routing; "tower" /
# "wide" / "wide64" (fp64 wide path for any input dtype) force a path where it applies
FCM_FORCE_PATH = ""


def make_fcm_ops(x: torch.Tensor, k: int, dtype: str = "fp64", m: float = 2.0,
                 nan_to_zero: bool = True, backend: str = "auto", distances: str = "x3"):
    """FCM tower for (dtype, K, D).  fp64 / fp32: the fused small-K*D kernel; from K = 64
    (fp32: and D = 64, fcm_f64_mfma) the fp64 f64-MFMA wide path with fused row statistics
    (fp32 rows promoted -- faster than the fp32 SIMT tower and fp64-accurate, like the
    reference's fp64 FCM, `scripts/distribuitedClustering.py:112-137`); below it the exact
    difference-form SIMT tower up to D = 256 and the wide tower above.
    bf16 (and fp8): the MFMA towers (fp32 rows split into bf16 hi/lo, bf16x3 distances,
    memberships in fp32, W = u^m rounded to bf16 for the W^T X MFMAs; centroid error
    ~1e-3 of max|c| against the fp64 oracle, FCM_PRECISION) for 16 < D <= 1024, K >= 32;
    other shapes fall back to the exact fp32 towers.  ``distances`` (ClusterConfig
    .fcm_distances): 'one' = one-product distances + two-nearest fix-up in both passes
    (D >= 64), 'x3' = bf16x3 distances in the accumulate pass."""
    d = x.shape[1]
    mfma = dtype in ("bf16", "fp8")
    if mfma:
        dtype = "fp32"  # memberships and rows in fp32; the distances on the matrix cores
    if not use_native(x.device, backend):
        return TorchFCM(x, k, dtype, m, nan_to_zero)
    tdt = torch.float64 if dtype == "fp64" else torch.float32
    if _native.require().fcm_small_supported(tdt, k, d):
        return HipSmallFCM(x, k, dtype, m, nan_to_zero)
    if mfma and d > 16 and k >= FCM_MFMA_MIN_K:
        if fcm_mfma_dim(d) is not None:
            ops = HipMfmaFCM(x, k, m, nan_to_zero)
            ops.one_product = distances == "one"
            return ops
        if fcm_mfma_wide_dim(d) is not None:
            return HipMfmaWideFCM(x, k, m, nan_to_zero)
    force = FCM_FORCE_PATH  # A/B only (bench.py --fcm-path): tower | wide | wide64
    if force == "tower" and d <= 256:
        return HipTowerFCM(x, k, dtype, m, nan_to_zero)
    if force in ("wide", "wide64"):
        return HipWideFCM(x, k, "fp64" if force == "wide64" else dtype, m, nan_to_zero)
    if fcm_f64_mfma(k, d, dtype):
        # fp64 on the f64 matrix cores (fused row statistics); fp32 rows are promoted to it
        # where that beats the fp32 SIMT tower (and is more accurate)
        return HipWideFCM(x, k, "fp64", m, nan_to_zero)
    if d <= 256:
        return HipTowerFCM(x, k, dtype, m, nan_to_zero)
    return HipWideFCM(x, k, dtype, m, nan_to_zero)


# Where fp32 / fp64 FCM run HipWideFCM's fused fp64 MFMA path instead of the SIMT towers
# (N=1M, m=2, ms/iter, profiles/fcm_route_r06f.txt):
#   D=32  K=32: fp64 tower 0.85 / f64-MFMA 1.23;  K=128: 1.63 / 1.45 (fp32 tower 1.08);
#         K=1024: 10.6 / 9.78 (fp32 tower 7.25)
#   D=128 K=64: 3.63 / 1.86 (fp32 tower 2.29);  K=128: 6.43 / 2.12 (4.12);  K=1024: 45.4 /
#         14.0 (28.2);  D=256 K=1024: 128 / 25.3 (66.5)
# fp64 from K = 64; fp32 (promoted) from K = 64 and D = 64 -- at D = 32 its SIMT tower wins
FCM_F64_MFMA_MIN_K = 64
FCM_F64_MFMA_MIN_D_FP32 = 64


def fcm_f64_mfma(k: int, d: int, dtype: str = "fp64") -> bool:
    if k < FCM_F64_MFMA_MIN_K:
        return False
    return dtype == "fp64" or d >= FCM_F64_MFMA_MIN_D_FP32
