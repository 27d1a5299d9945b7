"""Process-group runtime: one process per GPU, RCCL over xGMI (gloo on CPU).

Replaces the reference's in-graph replication + CPU parameter server
(`scripts/distribuitedClustering.py:84-148,193-263`): there every tower's
partial sums went device->host and were `tf.add_n`-ed on `/cpu:0` every
iteration.  Here each rank owns a contiguous row shard
(``np.array_split`` semantics, `:76,184`), keeps its partial sums on device and
the ranks combine them with ONE packed all-reduce per iteration; every rank then
finalises the (replicated) centroids itself, so no broadcast is needed.

Launch with ``torchrun --nproc-per-node G`` (``backend="nccl"`` is RCCL on
ROCm).  On a CPU-only host the same code runs with ``gloo``.
"""
from __future__ import annotations

import datetime
import os
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


def shard_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    """[start, end) of ``rank``'s rows under ``np.array_split(range(n), world)``.

    The first ``n % world`` shards get one extra row (`distribuitedClustering.py:76`).
    """
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


# exact cluster counts through an fp32 all-reduce: count = SPLIT * hi + lo with lo < SPLIT;
# both halves are integers below 2^24 per rank, so the fp32 sum over up to 4096 ranks is
# exact and counts stay exact up to 2^36 (ClusterConfig buffers with fp32 partial sums)
COUNT_SPLIT = 4096


def split_counts(c: torch.Tensor, hi: torch.Tensor, lo: torch.Tensor):
    """hi += c // SPLIT, lo += c % SPLIT for integer-valued counts ``c`` (any dtype)."""
    ci = c.to(torch.int64)
    hi.add_(torch.div(ci, COUNT_SPLIT, rounding_mode="floor").to(hi.dtype))
    lo.add_(torch.remainder(ci, COUNT_SPLIT).to(lo.dtype))


def join_counts(hi: torch.Tensor, lo: torch.Tensor) -> torch.Tensor:
    """Exact fp64 counts from the all-reduced halves."""
    return hi.double() * COUNT_SPLIT + lo.double()


def shard_sizes(n: int, world: int) -> List[int]:
    return [shard_bounds(n, world, r)[1] - shard_bounds(n, world, r)[0] for r in range(world)]


class Comm:
    """Thin handle over the default process group (or a single-process no-op)."""

    def __init__(self, device: torch.device, rank: int = 0, world_size: int = 1,
                 local_rank: int = 0, group=None, backend: str = "",
                 force_collectives: bool = False):
        self.device = device
        self.backend = backend
        self.rank = rank
        self.world_size = world_size
        self.local_rank = local_rank
        self.group = group
        # collectives are issued (not short-circuited) on more than one rank, or on a
        # world-1 process group when forced: TDC_FORCE_COLLECTIVES=1 runs every RCCL call
        # of the production path on a single GPU (tests/test_rccl_gpu.py)
        self.collective = world_size > 1 or force_collectives

    # ------------------------------------------------------------------ props
    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1

    @property
    def is_root(self) -> bool:
        return self.rank == 0

    def shard(self, n: int) -> Tuple[int, int]:
        return shard_bounds(n, self.world_size, self.rank)

    # ------------------------------------------------------------ collectives
    def allreduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self.collective:
            rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX,
                   "min": dist.ReduceOp.MIN}[op]
            dist.all_reduce(t, op=rop, group=self.group)
        return t

    def allreduce_bucketed_(self, flat: torch.Tensor, bucket_bytes: int = 0) -> torch.Tensor:
        """SUM all-reduce of a flat buffer, in one call or in ``bucket_bytes`` pieces.

        One call is the default and the fast path: RCCL already stripes a single
        all-reduce over its channels (one ring per xGMI link pair), so one call
        uses all 7 links of an MI355X; calls on one communicator run one after
        another on its stream, so buckets add a latency per call and never run
        "on separate links".  Buckets only bound the size of each call (e.g. to
        keep RCCL's staging buffers small next to a 201 MB K=65536 x D=768
        buffer); the large-K*D bandwidth win is :meth:`reduce_scatter_` +
        :meth:`all_gather_` (``ClusterConfig.comm_mode='rsag'``).
        """
        if not self.collective:
            return flat
        nbytes = flat.numel() * flat.element_size()
        if bucket_bytes <= 0 or nbytes <= bucket_bytes:
            dist.all_reduce(flat, group=self.group)
            return flat
        per = max(1, bucket_bytes // flat.element_size())
        for s in range(0, flat.numel(), per):
            dist.all_reduce(flat[s:s + per], group=self.group)
        return flat

    def reduce_scatter_(self, out: torch.Tensor, flat: torch.Tensor) -> torch.Tensor:
        """SUM reduce-scatter: rank r receives block r of ``flat`` (``flat.numel() ==
        world * out.numel()``), summed over ranks."""
        if not self.collective:
            out.copy_(flat.view_as(out))
            return out
        dist.reduce_scatter_tensor(out, flat, group=self.group)
        return out

    def all_gather_(self, out: torch.Tensor, part: torch.Tensor) -> torch.Tensor:
        """``out`` = concatenation over ranks of ``part`` (``out.numel() == world *
        part.numel()``; ``part`` must not alias ``out``)."""
        if not self.collective:
            out.copy_(part.view_as(out))
            return out
        if out.dtype in (torch.float8_e4m3fn, torch.float8_e5m2):
            # a gather moves bytes: fp8 operand tables travel as uint8 (gloo has no fp8)
            out, part = out.view(torch.uint8), part.view(torch.uint8)
        dist.all_gather_into_tensor(out, part, group=self.group)
        return out

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.collective:
            dist.broadcast(t, src=src, group=self.group)
        return t

    def barrier(self):
        if self.collective:
            if self.device.type == "cuda" and self.backend == "nccl":
                dist.barrier(group=self.group, device_ids=[self.device.index])
            else:
                dist.barrier(group=self.group)

    def max_scalar(self, v: float) -> float:
        if not self.collective:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return float(t.item())

    def sum_scalar(self, v: float) -> float:
        if not self.collective:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=self.device)
        dist.all_reduce(t, group=self.group)
        return float(t.item())

    def all_gather_sizes(self, n_local: int) -> List[int]:
        if not self.collective:
            return [n_local]
        t = torch.zeros(self.world_size, dtype=torch.int64, device=self.device)
        t[self.rank] = n_local
        dist.all_reduce(t, group=self.group)
        return [int(v) for v in t.tolist()]

    def gather_rows_to_root(self, local: torch.Tensor) -> Optional[torch.Tensor]:
        """Concatenate every rank's rows on rank 0 (variable sizes; for outputs only)."""
        if not self.collective:
            return local
        sizes = self.all_gather_sizes(local.shape[0])
        mx = max(sizes)
        # gloo gathers host tensors only (GPU ranks over gloo: TDC_DIST_BACKEND=gloo)
        dev = torch.device("cpu") if self.backend == "gloo" else self.device
        buf = torch.zeros((mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=dev)
        buf[: local.shape[0]] = local.to(dev)
        if self.rank == 0:
            bufs = [torch.empty_like(buf) for _ in range(self.world_size)]
            dist.gather(buf, gather_list=bufs, dst=0, group=self.group)
            return torch.cat([b[:s] for b, s in zip(bufs, sizes)])
        dist.gather(buf, dst=0, group=self.group)
        return None


_COMM: Optional[Comm] = None


def init_comm(device_type: Optional[str] = None, timeout_s: float = 600.0,
              debug: bool = False) -> Comm:
    """Initialise (once) from torchrun's env:// variables.

    device_type: 'cuda' | 'cpu' | None (auto: cuda if visible).
    timeout_s:   collective timeout: a hung peer fails the run instead of blocking it.
    debug:       collective-mismatch detection: ``TORCH_DISTRIBUTED_DEBUG=
                 DETAIL`` wraps the process group so every collective first checks that
                 all ranks issue the same op with the same shapes and dtypes (a rank that
                 diverges raises instead of deadlocking or corrupting a reduction).  Costs
                 an extra small collective per call: for tests and debugging runs.
    """
    global _COMM
    if _COMM is not None:
        return _COMM
    if debug:
        os.environ["TORCH_DISTRIBUTED_DEBUG"] = "DETAIL"
        dist.set_debug_level(dist.DebugLevel.DETAIL)  # the env is read once, at import
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    if device_type == "cuda":
        ndev = torch.cuda.device_count()
        dev_index = local_rank % max(1, ndev)
        torch.cuda.set_device(dev_index)
        device = torch.device("cuda", dev_index)
    else:
        device = torch.device("cpu")
    group = None
    # TDC_DIST_BACKEND=gloo runs GPU ranks over gloo (host-staged collectives): rehearses the
    # multi-rank GPU path with several ranks on ONE GPU, which RCCL does not allow
    backend = os.environ.get("TDC_DIST_BACKEND") or ("nccl" if device_type == "cuda" else "gloo")
    force = os.environ.get("TDC_FORCE_COLLECTIVES", "0") == "1"
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1 and "MASTER_PORT" not in os.environ:
            # a forced world-1 group (no launcher): any free local port
            import socket
            with socket.socket() as so:
                so.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(so.getsockname()[1])
        kw = dict(backend=backend, init_method="env://", world_size=world, rank=rank,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if device_type == "cuda" and backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    if dist.is_initialized():
        backend = str(dist.get_backend())
    _COMM = Comm(device, rank, world, local_rank, group,
                 backend if (world > 1 or force) else "", force_collectives=force)
    return _COMM


def local_comm(device: torch.device) -> Comm:
    """A single-rank communicator (no process group)."""
    return Comm(device, 0, 1, 0, None)


def destroy_comm():
    global _COMM
    if dist.is_initialized():
        dist.destroy_process_group()
    _COMM = None
