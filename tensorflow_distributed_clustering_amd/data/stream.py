"""Chunked data sources for streamed (larger-than-HBM) and mini-batch clustering.

Every source yields ``(global_row_start, chunk)`` where ``chunk`` is a device tensor
already in the kernel layout (``layout = (torch dtype, padded width)``):

* :class:`ResidentSource`  -- the shard is on the device; chunks are row views.
* :class:`HostSource`      -- the shard is in host memory (numpy array / NPZ memory map).
  A native :class:`RowStreamer` (csrc/loader.cpp) converts rows (f64/f32 -> bf16/f32/f64,
  zero-padded) into a ring of pinned buffers on worker threads; H2D copies run on a
  separate HIP stream into two device slots, so conversion, PCIe transfer and compute
  of consecutive chunks overlap.  This is what the reference attempted with
  ``tf.data`` (`notebooks/batching_tests.ipynb:353-378`) and never finished.
* :class:`SyntheticSource` -- Gaussian blobs generated chunk by chunk on the device
  (world-size invariant), e.g. N = 1e9 without ever materialising the dataset.
"""
from __future__ import annotations

from typing import Iterator, Optional, Tuple

import numpy as np
import torch

from .. import _native
from .synth import gaussian_blobs

Layout = Tuple[torch.dtype, int]


def to_layout(x: torch.Tensor, layout: Layout, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Copy/convert rows into ``layout`` (zero-padded columns)."""
    dt, width = layout
    if x.dtype == dt and x.shape[1] == width and x.is_contiguous() and out is None:
        return x
    if out is None:
        out = torch.zeros(x.shape[0], width, dtype=dt, device=x.device)
    elif x.shape[1] < width:
        out[:, x.shape[1]:].zero_()
    out[:, : x.shape[1]] = x
    return out


class ResidentSource:
    def __init__(self, x: torch.Tensor, layout: Layout, row_offset: int = 0):
        self.x = to_layout(x, layout)
        self.n_rows = self.x.shape[0]
        self.row_offset = row_offset
        self.layout = layout

    def chunks(self, chunk_rows: int) -> Iterator[Tuple[int, torch.Tensor]]:
        chunk_rows = chunk_rows or self.n_rows
        for s in range(0, self.n_rows, chunk_rows):
            yield self.row_offset + s, self.x[s:s + chunk_rows]

    def rows(self, idx: torch.Tensor) -> torch.Tensor:
        return self.x.index_select(0, idx)


class SyntheticSource:
    """Gaussian blobs produced on the device chunk by chunk (counter-based generator)."""

    def __init__(self, n_rows: int, d: int, n_centers: int, seed: int, row_offset: int,
                 layout: Layout, device, cluster_std: float = 1.0):
        self.n_rows, self.d, self.n_centers, self.seed = n_rows, d, n_centers, seed
        self.row_offset, self.layout, self.device = row_offset, layout, torch.device(device)
        self.cluster_std = cluster_std
        self._buf = None

    def _gen(self, start: int, rows: int) -> torch.Tensor:
        x = gaussian_blobs(rows, self.d, self.n_centers, seed=self.seed,
                           row_offset=self.row_offset + start, cluster_std=self.cluster_std,
                           dtype=self.layout[0], device=self.device)
        if self.layout[1] == self.d:
            return x
        if self._buf is None or self._buf.shape[0] < rows:
            self._buf = torch.zeros(rows, self.layout[1], dtype=self.layout[0], device=self.device)
        return to_layout(x, self.layout, self._buf[:rows])

    def chunks(self, chunk_rows: int) -> Iterator[Tuple[int, torch.Tensor]]:
        chunk_rows = chunk_rows or self.n_rows
        for s in range(0, self.n_rows, chunk_rows):
            yield self.row_offset + s, self._gen(s, min(chunk_rows, self.n_rows - s))


class HostSource:
    """Host-resident shard streamed through pinned memory by the native RowStreamer."""

    def __init__(self, x_host: np.ndarray, layout: Layout, device, row_offset: int = 0,
                 n_pinned: int = 3, n_threads: int = 8, resident_rows: int = 0):
        if x_host.dtype not in (np.float64, np.float32):
            x_host = np.ascontiguousarray(x_host, dtype=np.float32)
        if x_host.strides[1] != x_host.itemsize:
            x_host = np.ascontiguousarray(x_host)
        self.x = x_host  # keep the (memory-mapped) array alive while streaming
        self.n_rows, self.d = x_host.shape
        self.layout = layout
        self.device = torch.device(device)
        self.row_offset = row_offset
        self.n_pinned = max(2, n_pinned)
        dst_codes = {torch.bfloat16: 0, torch.float32: 1, torch.float64: 2}
        if layout[0] not in dst_codes:
            raise ValueError("HostSource streams to bf16, fp32 or fp64 layouts")
        dst_type = dst_codes[layout[0]]
        _native.require()
        ld = x_host.strides[0] // x_host.itemsize
        self.streamer = torch.classes.tdc.RowStreamer(
            int(x_host.ctypes.data), 0 if x_host.dtype == np.float64 else 1, self.n_rows, self.d,
            ld, dst_type, layout[1], n_threads)
        # hybrid residency: the first resident_rows rows are uploaded once and stay in HBM;
        # only the remainder streams every pass (data 1.5x HBM -> 1/3 of it crosses PCIe)
        self.resident_rows = int(min(max(0, resident_rows), self.n_rows)) if self.device.type == "cuda" else 0
        self._resident = None
        self.bytes_h2d = 0  # streamed (non-resident) bytes handed to the device so far

    def chunks(self, chunk_rows: int) -> Iterator[Tuple[int, torch.Tensor]]:
        chunk_rows = min(chunk_rows or self.n_rows, self.n_rows)
        dt, width = self.layout
        use_cuda = self.device.type == "cuda"
        pinned = [torch.empty(chunk_rows, width, dtype=dt, pin_memory=use_cuda)
                  for _ in range(self.n_pinned)]
        if not use_cuda:  # CPU ranks: the pinned slot is the chunk
            starts = list(range(0, self.n_rows, chunk_rows))
            for i, s in enumerate(starts):
                rows = min(chunk_rows, self.n_rows - s)
                slot = pinned[i % self.n_pinned]
                self.streamer.wait(self.streamer.submit(slot, s, rows))
                yield self.row_offset + s, slot[:rows]
            return
        R = self.resident_rows
        if R and self._resident is None:
            self._resident = torch.empty(R, width, dtype=dt, device=self.device)
            for s0 in range(0, R, chunk_rows):  # one-time upload through the same converter
                rows = min(chunk_rows, R - s0)
                self.streamer.wait(self.streamer.submit(pinned[0], s0, rows))
                self._resident[s0:s0 + rows].copy_(pinned[0][:rows])
            torch.cuda.current_stream(self.device).synchronize()
        for s0 in range(0, R, chunk_rows):
            yield self.row_offset + s0, self._resident[s0:min(R, s0 + chunk_rows)]
        if R >= self.n_rows:
            return
        devbuf = [torch.empty(chunk_rows, width, dtype=dt, device=self.device) for _ in range(2)]
        copy_stream = torch.cuda.Stream(device=self.device)
        compute = torch.cuda.current_stream(self.device)
        starts = list(range(R, self.n_rows, chunk_rows))
        tickets = {}
        h2d_done = [None] * self.n_pinned
        slot_free = [None, None]

        def submit(i):
            s = starts[i]
            j = i % self.n_pinned
            if h2d_done[j] is not None:
                h2d_done[j].synchronize()  # the DMA that read this pinned slot has finished
            tickets[i] = self.streamer.submit(pinned[j], s, min(chunk_rows, self.n_rows - s))

        for i in range(min(self.n_pinned, len(starts))):
            submit(i)
        for i, s in enumerate(starts):
            rows = min(chunk_rows, self.n_rows - s)
            self.streamer.wait(tickets.pop(i))
            j, b = i % self.n_pinned, i % 2
            with torch.cuda.stream(copy_stream):
                if slot_free[b] is not None:
                    copy_stream.wait_event(slot_free[b])  # consumer finished the old chunk
                devbuf[b][:rows].copy_(pinned[j][:rows], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(copy_stream)
            h2d_done[j] = ev
            compute.wait_event(ev)
            self.bytes_h2d += rows * width * devbuf[b].element_size()
            yield self.row_offset + s, devbuf[b][:rows]
            done = torch.cuda.Event()
            done.record(compute)
            slot_free[b] = done
            if i + self.n_pinned < len(starts):
                submit(i + self.n_pinned)
        torch.cuda.current_stream(self.device).synchronize()


class PlainHostSource(HostSource):
    """Host-resident fp32 / fp64 rows streamed as they are (no bf16 conversion): the same
    pinned ring, worker-thread row copies and copy-stream H2D as :class:`HostSource`
    (the fp64 kernels' layout is the source's own rows)."""

    def __init__(self, x_host: np.ndarray, layout: Layout, device, row_offset: int = 0,
                 n_pinned: int = 3, n_threads: int = 8, resident_rows: int = 0):
        if layout[0] not in (torch.float32, torch.float64):
            raise ValueError("PlainHostSource streams fp32 / fp64 rows")
        super().__init__(x_host, layout, device, row_offset, n_pinned, n_threads, resident_rows)

    def rows(self, idx: torch.Tensor) -> torch.Tensor:
        sel = torch.from_numpy(np.ascontiguousarray(self.x[idx.cpu().numpy()]))
        return sel.to(self.layout[0]).to(self.device)


def plan_chunk_rows(n_rows: int, row_bytes: int, k: int, d: int, device,
                    budget_gb: float = 0.0, reserve_frac: float = 0.15,
                    per_row_extra: int = 16, extra_fixed: int = 0) -> int:
    """Rows of one resident chunk that fit the HBM budget (0 = the whole shard fits).

    per_row_extra covers labels (4 B), the counting-sort permutation (4 B) and the
    min-distance buffer (4 B) per row.  MI355X has 288 GB of HBM3E per GPU; the budget
    defaults to what ``torch.cuda.mem_get_info`` reports free.
    """
    device = torch.device(device)
    if budget_gb > 0:
        budget = budget_gb * (1 << 30)
    elif device.type == "cuda":
        free, _total = torch.cuda.mem_get_info(device)
        budget = free
    else:
        return 0
    budget *= (1.0 - reserve_frac)
    fixed = k * d * 16 + (64 << 20) + int(extra_fixed)
    per_row = row_bytes + per_row_extra
    if n_rows * per_row + fixed <= budget:
        return 0
    rows = int((budget - fixed) // (2 * per_row + row_bytes))  # 2 device slots + staging
    return max(1 << 16, (rows // 4096) * 4096)


def plan_resident_rows(n_rows: int, row_bytes: int, chunk_rows: int, k: int, d: int, device,
                       budget_gb: float = 0.0, reserve_frac: float = 0.15,
                       per_row_extra: int = 16, extra_fixed: int = 0) -> int:
    """Rows of a streamed shard that can stay resident in HBM next to the streaming
    buffers (2 device slots of chunk_rows) and the per-row work buffers of all rows."""
    device = torch.device(device)
    if device.type != "cuda":
        return 0
    if budget_gb > 0:
        budget = budget_gb * (1 << 30)
    else:
        budget, _ = torch.cuda.mem_get_info(device)
    budget *= (1.0 - reserve_frac)
    fixed = (k * d * 16 + (64 << 20) + 2 * chunk_rows * row_bytes + n_rows * per_row_extra
             + int(extra_fixed))
    return int(max(0, min(n_rows, (budget - fixed) // row_bytes)))
