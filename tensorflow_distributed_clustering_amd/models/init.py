"""Distributed centroid initialisation.

Reference variants:
* k-means++ via sklearn's private ``k_means_._init_centroids`` on the host, per batch
  (`scripts/distribuitedClustering.py:82,191`);
* first-K rows ``X[0:K]`` (`:325`; the CSV-era revision);
* K random rows without replacement (`ckpt/Testing Images-checkpoint.ipynb:290-291`).
* (new) k-means|| (Bahmani et al. 2012): O(5) data sweeps instead of K, for large K.

Here every method is *world-size invariant*: the chosen global row indices depend only
on ``seed`` and ``N``, and each rank contributes the rows it owns to one SUM all-reduce,
so a 1-GPU and an 8-GPU run start from bit-identical centroids.  k-means++ runs on the
device shards (distributed D^2 sampling: one all-reduce of per-rank potentials + one of
the candidate rows per step) instead of on a host copy of the whole dataset.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..parallel.dist import Comm


def floyd_sample(n: int, k: int, seed: int) -> List[int]:
    """k distinct integers from [0, n) in O(k) (Floyd's algorithm), order randomised."""
    if k > n:
        raise ValueError(f"cannot draw {k} distinct rows from {n}")
    rng = np.random.default_rng(seed)
    chosen = {}
    out = []
    for j in range(n - k, n):
        t = int(rng.integers(0, j + 1))
        if t in chosen:
            t = j
        chosen[t] = True
        out.append(t)
    rng.shuffle(out)
    return out


def gather_global_rows(x_local: torch.Tensor, row_offset: int, idx: Sequence[int],
                       comm: Comm, dtype=torch.float64) -> torch.Tensor:
    """Rows ``idx`` (global indices) of the sharded matrix, replicated on every rank."""
    d = x_local.shape[1]
    out = torch.zeros(len(idx), d, dtype=dtype, device=x_local.device)
    n_local = x_local.shape[0]
    if len(idx):
        gi = torch.as_tensor(list(idx), dtype=torch.int64)
        mine = (gi >= row_offset) & (gi < row_offset + n_local)
        if bool(mine.any()):
            pos = torch.nonzero(mine).flatten()
            rows = (gi[mine] - row_offset).to(x_local.device)
            out[pos.to(x_local.device)] = x_local.index_select(0, rows).to(dtype)
    comm.allreduce_(out)
    return out


def init_random(x_local, row_offset, n_global, k, comm, seed):
    idx = floyd_sample(n_global, k, seed)
    return gather_global_rows(x_local, row_offset, idx, comm)


def init_first_k(x_local, row_offset, n_global, k, comm, seed=0):
    if k > n_global:
        raise ValueError("K larger than the number of points")
    return gather_global_rows(x_local, row_offset, range(k), comm)


def _sqdist_to(x: torch.Tensor, c: torch.Tensor, chunk: int = 1 << 22) -> torch.Tensor:
    """||x_i - c_j||^2 for a handful of candidate rows c [T, D] -> [T, n] (fp32/fp64)."""
    out = torch.empty(c.shape[0], x.shape[0], dtype=c.dtype, device=x.device)
    cc = (c * c).sum(1)[:, None]
    for s in range(0, x.shape[0], chunk):
        xs = x[s:s + chunk].to(c.dtype)
        xx = (xs * xs).sum(1)[None, :]
        out[:, s:s + chunk] = (torch.addmm(cc, c, xs.t(), alpha=-2.0) + xx).clamp_min_(0)
    return out


def _native_kpp(x_local, wd, trials):
    """The N7 kernel applies to GPU shards (bf16/fp32/fp64 rows, candidates fit LDS)."""
    if x_local.device.type != "cuda" or trials > 16:
        return None
    if x_local.dtype not in (torch.bfloat16, torch.float32, torch.float64) or x_local.stride(1) != 1:
        return None
    if trials * x_local.shape[1] * (8 if wd == torch.float64 else 4) > 64 * 1024:
        return None
    from .. import _native
    return _native.require()


def init_kmeanspp(x_local, row_offset, n_global, k, comm: Comm, seed,
                  n_local_trials: Optional[int] = None, work_dtype=None):
    """Distributed greedy k-means++ (sklearn's variant: 2 + ln K trials per step).

    On a GPU shard each step is two passes of the N7 kernel (`csrc/kmeanspp.hip`): score
    all candidates in one sweep, then apply the winner; elsewhere the same step in torch."""
    if n_local_trials is None:
        n_local_trials = 2 + int(math.log(k))
    dev = x_local.device
    wd = work_dtype or (torch.float64 if x_local.dtype == torch.float64 or dev.type == "cpu"
                        else torch.float32)
    ops = _native_kpp(x_local, wd, n_local_trials)
    rng = np.random.default_rng(seed)
    n_local = x_local.shape[0]
    centers = torch.empty(k, x_local.shape[1], dtype=torch.float64, device=dev)
    first = int(rng.integers(0, n_global))
    centers[0] = gather_global_rows(x_local, row_offset, [first], comm)[0]
    pots_buf = torch.zeros(max(16, n_local_trials), dtype=torch.float64, device=dev)
    if ops is not None:
        closest = torch.full((n_local,), float("inf"), dtype=wd, device=dev)
        pots_buf.zero_()
        ops.kpp_step(x_local, centers[:1].to(wd).contiguous(), closest, 1, pots_buf)
        local_pot = pots_buf[:1].clone()
    else:
        closest = _sqdist_to(x_local, centers[:1].to(wd))[0]
        local_pot = closest.sum().double().reshape(1)
    for c in range(1, k):
        pots = torch.zeros(comm.world_size, dtype=torch.float64, device=dev)
        pots[comm.rank] = local_pot[0]
        comm.allreduce_(pots)
        pots_h = pots.cpu().numpy()
        total = float(pots_h.sum())
        if total <= 0.0:
            cand_idx = [int(v) for v in rng.integers(0, n_global, size=n_local_trials)]
        else:
            r = rng.random(n_local_trials) * total
            cum = np.cumsum(pots_h)
            owners = np.searchsorted(cum, r, side="right").clip(0, comm.world_size - 1)
            cand_idx = [0] * n_local_trials
            local_cs = None
            for t in range(n_local_trials):
                if owners[t] == comm.rank:
                    if local_cs is None:
                        local_cs = torch.cumsum(closest.double(), 0)
                    rr = r[t] - (cum[owners[t]] - pots_h[owners[t]])
                    li = int(torch.searchsorted(local_cs, torch.tensor([rr], dtype=torch.float64,
                                                                       device=dev)).item())
                    cand_idx[t] = row_offset + min(li, n_local - 1)
            ci = torch.tensor(cand_idx, dtype=torch.int64, device=dev)
            comm.allreduce_(ci)  # only the owner wrote a non-zero (owners differ per trial)
            cand_idx = [int(v) for v in ci.tolist()]
        cand = gather_global_rows(x_local, row_offset, cand_idx, comm)
        if ops is not None:
            tp = pots_buf[: len(cand_idx)]
            tp.zero_()
            ops.kpp_step(x_local, cand.to(wd).contiguous(), closest, 0, tp)
            tp = tp.clone()
            comm.allreduce_(tp)
            best = int(torch.argmin(tp).item())
            pots_buf.zero_()
            ops.kpp_step(x_local, cand[best:best + 1].to(wd).contiguous(), closest, 1, pots_buf)
            local_pot = pots_buf[:1].clone()
        else:
            dist = torch.minimum(_sqdist_to(x_local, cand.to(wd)), closest[None, :])
            tp = dist.double().sum(1)
            comm.allreduce_(tp)
            best = int(torch.argmin(tp).item())
            closest = dist[best].contiguous()
            local_pot = closest.sum().double().reshape(1)
        centers[c] = cand[best]
    return centers


# ------------------------------------------------------------------ k-means|| (Bahmani 2012)
def _hash_uniform(rows: torch.Tensor, seed: int, rnd: int) -> torch.Tensor:
    """Counter-based U[0,1) per GLOBAL row index: the sampling decision of a row does not
    depend on which rank owns it (world-size invariant)."""
    from ..data.synth import _mix32
    s = (int(seed) * 0x9E3779B1 + (rnd + 1) * 0x85EBCA6B) & 0xFFFFFFFF
    h = _mix32((rows * 0x27D4EB2F + s) & 0xFFFFFFFF)
    h2 = _mix32((h ^ 0x5BD1E995) & 0xFFFFFFFF)
    return ((h >> 8).double() * (1.0 / (1 << 24)) + (h2 >> 8).double() * (1.0 / (1 << 48)))


def _min_sqdist(x: torch.Tensor, c: torch.Tensor, chunk: int = 1 << 16):
    """(min_j ||x_i - c_j||^2, argmin) over a candidate set via chunked GEMM (fp32/fp64)."""
    wd = torch.float64 if (x.dtype == torch.float64 or x.device.type == "cpu") else torch.float32
    cw = c.to(wd)
    cc = (cw * cw).sum(1)[None, :]
    md = torch.empty(x.shape[0], dtype=wd, device=x.device)
    lab = torch.empty(x.shape[0], dtype=torch.int64, device=x.device)
    step = max(1, min(chunk, (1 << 28) // max(1, c.shape[0])))
    for s0 in range(0, x.shape[0], step):
        xs = x[s0:s0 + step].to(wd)
        d = torch.addmm(cc, xs, cw.t(), alpha=-2.0).add_((xs * xs).sum(1)[:, None])
        m, a = d.min(1)
        md[s0:s0 + step] = m.clamp_min_(0)
        lab[s0:s0 + step] = a
    return md, lab


def _gather_varlen(comm: Comm, local: torch.Tensor) -> torch.Tensor:
    """Concatenate every rank's 1-D int64 tensor (rank order), replicated."""
    sizes = comm.all_gather_sizes(int(local.numel()))
    total = int(sum(sizes))
    out = torch.zeros(total, dtype=torch.int64, device=comm.device)
    off = int(sum(sizes[: comm.rank]))
    out[off:off + local.numel()] = local.to(comm.device)
    comm.allreduce_(out)
    return out


def weighted_kmeanspp(c: torch.Tensor, w: torch.Tensor, k: int, seed: int,
                      lloyd_iters: int = 10) -> torch.Tensor:
    """k-means++ on a small weighted point set, then a few weighted Lloyd steps
    (the recluster step of k-means||; Spark MLlib's LocalKMeans does the same)."""
    rng = np.random.default_rng(seed)
    m = c.shape[0]
    c = c.double()
    w = w.double()
    trials = 2 + int(math.log(k))
    centers = torch.empty(k, c.shape[1], dtype=torch.float64, device=c.device)
    p0 = (w / w.sum()).cpu().numpy()
    first = int(rng.choice(m, p=p0))
    centers[0] = c[first]
    closest = ((c - c[first]) ** 2).sum(1)
    for j in range(1, k):
        pot = (w * closest)
        tot = float(pot.sum())
        if tot <= 0:
            cand = rng.integers(0, m, size=trials)
        else:
            cum = torch.cumsum(pot, 0).cpu().numpy()
            cand = np.searchsorted(cum, rng.random(trials) * tot, side="right").clip(0, m - 1)
        cd = torch.cdist(c, c[torch.as_tensor(cand, device=c.device)]) ** 2  # [m, T]
        nd = torch.minimum(cd, closest[:, None])
        best = int((w[:, None] * nd).sum(0).argmin())
        centers[j] = c[int(cand[best])]
        closest = nd[:, best]
    for _ in range(lloyd_iters):
        lab = torch.cdist(c, centers).argmin(1)
        s = torch.zeros_like(centers).index_add_(0, lab, c * w[:, None])
        n = torch.zeros(k, dtype=torch.float64, device=c.device).index_add_(0, lab, w)
        nz = n > 0
        centers[nz] = s[nz] / n[nz, None]
    return centers


# Greedy k-means++ is K dependent sweeps over the shard (~3 kernels + 4 small collectives
# per centre); above ClusterConfig.kpp_max_k (default 2048), init='kmeans++' runs the
# sampled k-means|| below instead.  K = 65536 greedy would be ~131K full sweeps -- hours.
KPP_MAX_K = 2048
# k-means|| on a uniform sample of this many rows per centre (sampled mode)
KPAR_SAMPLE_PER_K = 8
# greedy k-means++ sweeps a uniform sample of max(KPP_SAMPLE_MIN, kpp_sample_per_k * K)
# rows when the data has more than 4x that many (K sweeps of 100M rows at K = 1024 took
# 76 s on one MI355X; of the 262K-row sample, well under a second).
# ClusterConfig.kpp_sample_per_k = 0: always sweep the full shards.
KPP_SAMPLE_MIN = 50_000
KPP_SAMPLE_PER_K = 256
# weighted k-means++ recluster up to this many centres; above it the K centres are drawn
# from the candidates by weight without replacement (Python-level greedy is O(K) steps)
RECLUSTER_MAX_K = 2048


def init_kmeans_parallel(x_local, row_offset, n_global, k, comm: Comm, seed,
                         rounds: int = 5, oversample: float = 2.0, sample: int = 0):
    """Scalable k-means++ ("k-means||"): ``rounds`` passes that each keep every point
    with probability min(1, l d^2 / phi) (l = oversample*K), then weighted k-means++ on
    the ~l*rounds candidates.  O(rounds) sweeps over the data instead of K, and each pass
    is one chunked GEMM + one all-reduce.

    ``sample`` > 0 (large K): the rounds run on a uniform world-invariant sample of that
    many rows, replicated on every rank (one gather), with 2 rounds at l = K, and the K
    centres are drawn from the candidates by cluster mass (RECLUSTER_MAX_K) -- the whole
    seeding of K = 65536 is a few GEMM passes over a 0.5M-row sample."""
    if sample and sample < n_global:
        idx = floyd_sample(n_global, sample, seed + 31)
        xs = gather_global_rows(x_local, row_offset, idx, comm,
                                dtype=torch.float32 if x_local.device.type == "cuda"
                                else torch.float64)
        from ..parallel.dist import local_comm
        return init_kmeans_parallel(xs, 0, sample, k, local_comm(xs.device), seed,
                                    rounds=min(rounds, 2), oversample=min(oversample, 1.0))
    dev = x_local.device
    n_local = x_local.shape[0]
    rows = torch.arange(row_offset, row_offset + n_local, dtype=torch.int64, device=dev)
    l = oversample * k
    C = gather_global_rows(x_local, row_offset, floyd_sample(n_global, 1, seed), comm)
    md, _ = _min_sqdist(x_local, C)
    for rnd in range(rounds):
        phi = comm.sum_scalar(float(md.double().sum()))
        if phi <= 0:
            break
        u = _hash_uniform(rows, seed, rnd)
        pick = rows[u < (l * md.double() / phi)]
        idx = _gather_varlen(comm, pick)
        if idx.numel() == 0:
            continue
        newc = gather_global_rows(x_local, row_offset, idx.tolist(), comm)
        C = torch.cat([C, newc])
        nd, _ = _min_sqdist(x_local, newc)
        md = torch.minimum(md, nd)
    if C.shape[0] <= k:
        extra = floyd_sample(n_global, k, seed + 17)[: k - C.shape[0]]
        return torch.cat([C, gather_global_rows(x_local, row_offset, extra, comm)])
    _, lab = _min_sqdist(x_local, C)
    w = torch.bincount(lab, minlength=C.shape[0]).double()
    comm.allreduce_(w)
    if k > RECLUSTER_MAX_K:
        # K centres from the candidates by cluster mass, without replacement (seeded,
        # on the host so every rank draws the same set)
        g = torch.Generator().manual_seed(int(seed) + 101)
        wp = w.cpu() + 1e-12
        pick = torch.multinomial(wp, k, replacement=False, generator=g)
        return C[pick.to(C.device)].double()
    return weighted_kmeanspp(C, w, k, seed)


def _note(comm: Comm, msg: str):
    if comm.is_root:
        print(f"[init] {msg}", flush=True)


def init_centers(method: str, x_local: torch.Tensor, row_offset: int, n_global: int, k: int,
                 comm: Comm, seed: int = 0, given: Optional[torch.Tensor] = None,
                 kpp_max_k: int = KPP_MAX_K, kpp_sample_per_k: int = KPP_SAMPLE_PER_K,
                 kpp_sample_min: int = KPP_SAMPLE_MIN) -> torch.Tensor:
    """[K, D] float64 on the shard's device, identical on every rank.

    init='kmeans++' is exact greedy k-means++ over all rows only while K <= kpp_max_k and
    N <= 4 * max(kpp_sample_min, kpp_sample_per_k * K); otherwise it seeds on a uniform
    world-invariant sample (greedy k-means++ on the sample, or sampled k-means|| above
    kpp_max_k).  Either approximation is logged on the root rank."""
    if given is None and method != "given" and k > n_global:
        raise ValueError(f"K={k} is larger than the number of points N={n_global}")
    if given is not None or method == "given":
        if given is None:
            raise ValueError("init='given' needs init_centers")
        g = torch.as_tensor(np.asarray(given), dtype=torch.float64).to(x_local.device)
        if g.shape != (k, x_local.shape[1]):
            raise ValueError(f"init_centers must be [{k}, {x_local.shape[1]}], got {tuple(g.shape)}")
        return g
    if method == "random":
        return init_random(x_local, row_offset, n_global, k, comm, seed)
    if method == "first_k":
        return init_first_k(x_local, row_offset, n_global, k, comm, seed)
    if method == "kmeans++" and k <= kpp_max_k:
        m = max(kpp_sample_min, kpp_sample_per_k * k)
        if kpp_sample_per_k > 0 and n_global > 4 * m:
            # world-invariant uniform sample, replicated; greedy seeding on it
            _note(comm, f"kmeans++ seeds on a uniform sample of {m} of {n_global} rows "
                        f"(kpp_sample_per_k={kpp_sample_per_k}; 0 = all rows)")
            idx = floyd_sample(n_global, m, seed + 1)
            xs = gather_global_rows(x_local, row_offset, idx, comm,
                                    dtype=torch.float32 if x_local.device.type == "cuda"
                                    and x_local.dtype != torch.float64 else torch.float64)
            from ..parallel.dist import local_comm
            return init_kmeanspp(xs, 0, m, k, local_comm(xs.device), seed)
        return init_kmeanspp(x_local, row_offset, n_global, k, comm, seed)
    if method in ("kmeans++", "kmeans||"):
        sample = KPAR_SAMPLE_PER_K * k if k > kpp_max_k else 0
        if sample and sample < n_global:
            _note(comm, f"{method} with K={k} > kpp_max_k={kpp_max_k}: sampled k-means|| on "
                        f"{sample} of {n_global} rows, centres drawn by cluster mass")
        return init_kmeans_parallel(x_local, row_offset, n_global, k, comm, seed,
                                    sample=min(sample, n_global) if sample else 0)
    raise ValueError(f"unknown init {method!r}")


# ------------------------------------------------------------------ chunk sources
def _source_rows(source, local_idx, d: int) -> torch.Tensor:
    """float64 rows (local indices) of a chunk source, on the source's device."""
    from ..data.stream import HostSource, PlainHostSource, ResidentSource, SyntheticSource
    from ..data.synth import gaussian_blob_rows
    if isinstance(source, ResidentSource):
        idx = torch.as_tensor(local_idx, dtype=torch.int64, device=source.x.device)
        return source.x.index_select(0, idx)[:, :d].double()
    if isinstance(source, (HostSource, PlainHostSource)):
        rows = np.asarray(source.x[np.asarray(local_idx, dtype=np.int64)], dtype=np.float64)
        return torch.from_numpy(rows).to(source.device)
    if isinstance(source, SyntheticSource):
        g = [source.row_offset + int(i) for i in local_idx]
        return gaussian_blob_rows(g, d, source.n_centers, source.seed, source.cluster_std,
                                  dtype=torch.float64, device=source.device)
    raise TypeError(f"unsupported source {type(source).__name__}")


def gather_rows_from_source(source, row_offset: int, idx, comm: Comm, d: int) -> torch.Tensor:
    """Global rows ``idx`` of a sharded chunk source, replicated on every rank."""
    dev = comm.device
    out = torch.zeros(len(idx), d, dtype=torch.float64, device=dev)
    n_local = int(source.n_rows)
    pos, loc = [], []
    for p, g in enumerate(idx):
        if row_offset <= g < row_offset + n_local:
            pos.append(p)
            loc.append(g - row_offset)
    if pos:
        out[torch.as_tensor(pos, device=dev)] = _source_rows(source, loc, d).to(dev)
    comm.allreduce_(out)
    return out


def init_centers_from_source(method: str, source, row_offset: int, n_global: int, k: int,
                             comm: Comm, seed: int = 0, given=None, d: int = None,
                             rows=None, kpp_max_k: int = KPP_MAX_K,
                             kpp_sample_per_k: int = KPP_SAMPLE_PER_K,
                             kpp_sample_min: int = KPP_SAMPLE_MIN) -> torch.Tensor:
    """Init for streamed / generated shards (rows are gathered from the source).

    k-means++ on a source that is not device-resident runs on a uniform random sample of
    max(kpp_sample_min, kpp_sample_per_k * k) rows (replicated), the standard sample-based
    seeding for data that cannot be swept K times.  kpp_sample_per_k = 0 ("always the full
    data", ClusterConfig) gathers EVERY row onto each device: only for shards that fit.
    """
    if rows is not None:
        return gather_rows_from_source(source, row_offset, rows, comm, d)
    if given is not None or method == "given":
        g = torch.as_tensor(np.asarray(given), dtype=torch.float64).to(comm.device)
        if g.shape != (k, d):
            raise ValueError(f"init_centers must be [{k}, {d}], got {tuple(g.shape)}")
        return g
    if k > n_global:
        raise ValueError(f"K={k} is larger than the number of points N={n_global}")
    if method == "random":
        return gather_rows_from_source(source, row_offset, floyd_sample(n_global, k, seed), comm, d)
    if method == "first_k":
        return gather_rows_from_source(source, row_offset, range(k), comm, d)
    if method in ("kmeans++", "kmeans||"):
        m = n_global if kpp_sample_per_k <= 0 else \
            min(n_global, max(kpp_sample_min, kpp_sample_per_k * k))
        if m < n_global:
            _note(comm, f"{method} on a streamed shard seeds on a uniform sample of {m} of "
                        f"{n_global} rows")
        sample = gather_rows_from_source(source, row_offset, floyd_sample(n_global, m, seed + 1),
                                         comm, d)
        from ..parallel.dist import local_comm
        return init_centers(method, sample, 0, m, k, local_comm(sample.device), seed,
                            kpp_max_k=kpp_max_k, kpp_sample_per_k=0)
    raise ValueError(f"unknown init {method!r}")
