"""Frozen run configuration threaded through every layer.

The reference hard-codes its knobs: fixed iteration count with no tolerance
(`scripts/distribuitedClustering.py:163,277`), fuzzifier ``m := D``
(`:97,121,129`), k-means++ init (`:82,191`), NaN on empty clusters (`:240,248`).
Here each of those is an explicit field whose *default* is the correct
semantics and whose ``compat`` value reproduces the reference behaviour.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass
from typing import Optional

METHODS = ("distributedKMeans", "distributedFuzzyCMeans", "miniBatchKMeans")
DTYPES = ("fp64", "fp32", "bf16", "fp8")
INITS = ("random", "first_k", "kmeans++", "kmeans||", "given")
EMPTY_POLICIES = ("keep", "nan", "nan_any", "reseed", "zero")
BACKENDS = ("auto", "hip", "torch")
ALGORITHMS = ("lloyd", "bounded")
COMM_MODES = ("auto", "allreduce", "rsag")
UPDATE_MODES = ("auto", "full", "delta")
EXACT_ASSIGN = ("auto", "mfma", "simt")
FCM_DISTANCES = ("one", "x3")


@dataclass(frozen=True)
class ClusterConfig:
    """All knobs of one clustering run.

    n_clusters      K
    max_iter        fixed iteration budget (reference: ``--n_max_iters``)
    tol             stop when max centroid shift^2 <= tol (0 = run all iters,
                    the reference behaviour, `distribuitedClustering.py:163`)
    dtype           compute dtype of the distance kernel. bf16/fp8 use MFMA; fp32/fp64
                    K-Means (16 < D <= 1024) runs bf16x3 MFMA scores with an exact
                    re-check of every row the error bound cannot certify, so its labels
                    are the exact argmin of that dtype (``exact_assign='simt'``: the
                    difference-form SIMT tiles instead); FCM fp32/fp64 use exact
                    difference-form towers.
    init            centroid init (reference script: k-means++; CSV era: first-K)
    fuzzifier       FCM m. ``None`` = compat value D (`:121,129`).
    fcm_nan_to_zero compat: membership NaN (point on a centroid) -> 0 (`:125-126`);
                    False gives the correct one-hot membership.
    fcm_distances   bf16 FCM on the matrix cores (D >= 64): 'x3' (default) runs bf16x3
                    distances (16 of fp32's 24 mantissa bits per operand) in both passes;
                    'one' runs ONE bf16 product per distance with each row's two nearest
                    centroids corrected to bf16x3 (0.8x the step at fcm10m, but wrong where a
                    third centroid sits inside the one-product error of a tight blob: on the
                    fcm10m data 4.0e-2 ('one') vs 3.1e-5 ('x3') of max|c| against the fp64
                    oracle, profiles/bench_fcm10m_*_std025_r06h).
    empty_cluster   'keep' (default) | 'nan' (globally empty -> NaN, the segment-sum
                    notebook) | 'nan_any' (empty on ANY rank -> NaN, the script's
                    reduce_mean poisoning) | 'reseed' | 'zero'
    backend         'hip' native kernels, 'torch' reference ops, 'auto'
    deterministic   ordered per-block reduction instead of float atomics
    chunk_rows      rows per streamed chunk (0 = whole shard resident)
    hbm_budget_gb   planner budget per GPU (MI355X has 288 GB)
    checkpoint_*    periodic centroid checkpoints / resume (reference: none)
    algorithm       'lloyd' | 'bounded' (exact Lloyd that re-assigns only the rows its
                    Hamerly bounds cannot settle; resident bf16 MFMA path, else Lloyd)
    comm_mode       partial-sum reduction: 'allreduce' (one packed all-reduce, every rank
                    finalises all K), 'rsag' (reduce-scatter -> each rank finalises K/G
                    centroids and preps their assign operands -> all-gather of the
                    operands), 'auto' (rsag when the sums buffer >= 32 MiB and G > 1)
    bucket_kb       split the all-reduce into calls of this many KiB (0: one call)
    warmup          one discarded step before the timer starts (first-launch code-object
                    load and grid sizing go to setup_time).  The reference's
                    computation_time includes its first sess.run
                    (`distribuitedClustering.py:164-166`): set False for like-for-like
    kgroup_bytes    wide-D / fp8 assign: centroid bytes per K-group (0: one group)
    kpp_max_k       init='kmeans++' above this K seeds with sampled k-means|| instead of
                    greedy k-means++ (K dependent sweeps would take hours at K=65536)
    kpp_sample_per_k greedy k-means++ runs on a uniform world-invariant sample of
                    max(kpp_sample_min, kpp_sample_per_k * K) rows when N is over 4x that
                    (0: always the full data -- for a streamed / generated source that
                    gathers every row onto each device).  The root rank logs whenever a
                    sample is used.
    update          Lloyd centroid update: 'full' re-sums every row each step; 'delta' keeps
                    fp64 per-cluster totals and each step moves only the rows whose label
                    changed (+x into the new, -x out of the old cluster; same fixed points,
                    models/kmeans.py); 'auto' = delta where supported (resident shard, native
                    sorted/LDS update or the torch ops, K <= 65536, keep/nan/zero policies)
    delta_refresh   delta update: recompute the totals from every row each this many steps
                    (0: never); a step after one that moved more than delta_theta * N rows
                    is a full step too (the choice is made on the device)
    """

    n_clusters: int
    max_iter: int = 20
    tol: float = 0.0
    dtype: str = "bf16"
    init: str = "random"
    seed: int = 0
    fuzzifier: Optional[float] = None
    fcm_nan_to_zero: bool = True
    fcm_distances: str = "x3"
    empty_cluster: str = "keep"
    backend: str = "auto"
    deterministic: bool = False
    chunk_rows: int = 0
    hbm_budget_gb: float = 0.0
    compute_inertia: bool = True
    label_pass: bool = True
    batch_size: int = 0  # mini-batch K-Means: rows per rank per step
    log_every: int = 0
    checkpoint_path: str = ""   # NPZ written by rank 0 (utils/checkpoint.py)
    checkpoint_every: int = 0   # iterations between checkpoints (0: final only)
    resume: bool = False        # continue from checkpoint_path if it exists
    max_oom_retries: int = 4    # setup OOM -> halve the streamed chunk and retry
    graph: bool = False         # replay each Lloyd step from a captured hipGraph
    spherical: bool = False     # cosine / spherical K-Means: unit rows, unit centroids
    algorithm: str = "lloyd"    # 'bounded': Lloyd with Hamerly bounds (models/bounded.py)
    fp8_recheck: float = 0.0    # fp8: exact re-check of near ties (relative margin; 0 = off)
    comm_mode: str = "auto"     # 'allreduce' | 'rsag' | 'auto' (parallel/dist.py)
    bucket_kb: int = 0          # all-reduce bucket size (0: one call per iteration)
    oom_recovery: bool = True   # mid-run OOM on any rank -> roll back one step, go streamed
    warmup: bool = True         # discarded first step before the timed loop (see above)
    kgroup_bytes: int = 0       # wide-D / fp8 assign K-group size in bytes (0: one group)
    kpp_max_k: int = 2048       # greedy k-means++ up to this K, sampled k-means|| above
    kpp_sample_per_k: int = 256 # greedy k-means++ sample rows per centre (0: full data)
    kpp_sample_min: int = 50_000  # ... and at least this many rows
    update: str = "auto"        # 'auto' | 'full' | 'delta' (Lloyd centroid update)
    delta_refresh: int = 32     # delta update: full re-sum every this many steps (0: never)
    delta_theta: float = 0.4    # ... and after a step that moved more than this share of rows
    exact_assign: str = "auto"  # fp32/fp64 K-Means assign: 'auto'/'mfma' bf16x3 + exact re-check, 'simt'

    def __post_init__(self):
        if self.n_clusters <= 0:
            raise ValueError(f"n_clusters must be positive, got {self.n_clusters}")
        if self.max_iter < 0:
            raise ValueError("max_iter must be >= 0")
        if self.dtype not in DTYPES:
            raise ValueError(f"dtype must be one of {DTYPES}, got {self.dtype!r}")
        if self.init not in INITS:
            raise ValueError(f"init must be one of {INITS}, got {self.init!r}")
        if self.empty_cluster not in EMPTY_POLICIES:
            raise ValueError(f"empty_cluster must be one of {EMPTY_POLICIES}")
        if self.backend not in BACKENDS:
            raise ValueError(f"backend must be one of {BACKENDS}")
        if self.algorithm not in ALGORITHMS:
            raise ValueError(f"algorithm must be one of {ALGORITHMS}")
        if self.comm_mode not in COMM_MODES:
            raise ValueError(f"comm_mode must be one of {COMM_MODES}")
        if self.update not in UPDATE_MODES:
            raise ValueError(f"update must be one of {UPDATE_MODES}")
        if self.fcm_distances not in FCM_DISTANCES:
            raise ValueError(f"fcm_distances must be one of {FCM_DISTANCES}")
        if self.exact_assign not in EXACT_ASSIGN:
            raise ValueError(f"exact_assign must be one of {EXACT_ASSIGN}")
        if self.delta_refresh < 0 or not (0.0 <= self.delta_theta <= 1.0):
            raise ValueError("delta_refresh must be >= 0 and delta_theta in [0, 1]")

    def replace(self, **kw) -> "ClusterConfig":
        return dataclasses.replace(self, **kw)

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)
