"""Serving: assign new points to fitted centroids at high throughput / low latency.

The reference only labels the points it was fitted on (the per-iteration label pass,
`scripts/distribuitedClustering.py:255,282`); a deployed clustering model mostly answers
"which cluster is this point in" for fresh traffic.  :class:`ClusterPredictor` keeps the
centroid operands of the assignment kernel prepared once (bf16 ``-2c`` + ``||c||^2`` for
the MFMA kernel, fp8 block-scaled operands, or exact fp32/fp64 centroids) and reuses
per-batch-size input / output buffers, so a request is one kernel launch (plus a layout
copy when the caller's rows are not already in the kernel layout).  For a fixed batch
size, :meth:`ClusterPredictor.capture` records the assignment into a hipGraph that
:meth:`predict` replays after the layout copy.

    pred = ClusterPredictor(km.result_.centers, dtype="bf16", device="cuda")
    labels = pred.predict(x)                 # int32 [B]
    labels, d2 = pred.predict(x, return_distance=True)
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import numpy as np
import torch

from .ops import make_lloyd_ops


class ClusterPredictor:
    """Nearest-centroid assignment against a fixed centroid set (one device)."""

    def __init__(self, centers, dtype: str = "bf16", device=None, backend: str = "auto"):
        c = torch.as_tensor(np.asarray(centers) if not torch.is_tensor(centers) else centers)
        if c.dim() != 2:
            raise ValueError("centers must be [K, D]")
        dev = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
            else torch.device("cpu"))
        self.k, self.d = int(c.shape[0]), int(c.shape[1])
        self.device = dev
        self.dtype = dtype
        probe = torch.zeros(1, self.d, dtype=torch.float32, device=dev)
        self.local = make_lloyd_ops(probe, self.k, dtype, backend)
        self.C = c.to(dev, self.local.c_dtype).contiguous()
        self.local.prepare(self.C)
        self.layout = tuple(self.local.layout)
        self._bufs: Dict[int, Tuple[torch.Tensor, torch.Tensor, torch.Tensor]] = {}
        self._graphs: Dict[int, torch.cuda.CUDAGraph] = {}

    @property
    def backend(self) -> str:
        return self.local.name

    # ------------------------------------------------------------------ buffers
    def _buffers(self, n: int):
        b = self._bufs.get(n)
        if b is None:
            dt, width = self.layout
            xin = torch.zeros(n, width, dtype=dt, device=self.device)
            lab = torch.empty(n, dtype=torch.int32, device=self.device)
            mdt = torch.float64 if self.local.c_dtype == torch.float64 else torch.float32
            md = torch.empty(n, dtype=mdt, device=self.device)
            b = self._bufs[n] = (xin, lab, md)
        return b

    def _in_layout(self, x: torch.Tensor) -> bool:
        dt, width = self.layout
        return x.dtype == dt and x.dim() == 2 and x.shape[1] == width and x.is_contiguous()

    def _run(self, x: torch.Tensor, lab, md, want_dist: bool):
        self.local.bind(x).assign(self.C, lab, md if want_dist else None)

    # ------------------------------------------------------------------ API
    def predict(self, x, return_distance: bool = False, copy: bool = True):
        """Labels (int32 [B]) of the rows of ``x`` [B, D]; with ``return_distance`` also
        their squared distance to the chosen centroid (kernel arithmetic).  ``copy=False``
        returns the per-batch-size output buffers themselves (no extra kernel; valid until
        the next request of the same size)."""
        x = torch.as_tensor(x)
        if x.dim() != 2 or x.shape[1] != self.d:
            raise ValueError(f"expected [B, {self.d}] rows, got {tuple(x.shape)}")
        n = int(x.shape[0])
        if n == 0:
            e = torch.empty(0, dtype=torch.int32, device=self.device)
            return (e, torch.empty(0, device=self.device)) if return_distance else e
        xin, lab, md = self._buffers(n)
        x = x.to(self.device, non_blocking=True)
        g = self._graphs.get(n)
        if g is not None:
            xin[:, : self.d].copy_(x)  # (a no-op copy would still be a launch: always copy)
            g.replay()
        else:
            if self._in_layout(x):
                xin = x
            else:
                xin[:, : self.d].copy_(x)
            self._run(xin, lab, md, return_distance)
        if copy:
            lab, md = lab.clone(), (md.clone() if return_distance else md)
        if return_distance:
            return lab, md
        return lab

    def score(self, x) -> float:
        """Negative inertia of ``x`` against the centroids (sklearn convention)."""
        _, md = self.predict(x, return_distance=True)
        return -float(md.double().sum())

    def capture(self, batch_rows: int) -> "ClusterPredictor":
        """Record the assignment of ``batch_rows``-row requests (reading the size's layout
        buffer, writing labels AND distances into its output buffers) into a hipGraph;
        later :meth:`predict` calls of that size copy the rows into the layout buffer and
        replay it.  Worth it where the assignment is more than one launch (fp8: row
        quantiser + assignment; wide bf16: norms + assignment)."""
        if self.device.type != "cuda":
            raise RuntimeError("graph capture needs a GPU predictor")
        n = int(batch_rows)
        xin, lab, md = self._buffers(n)
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):  # warm-up outside capture (kernel attributes, allocations)
            self._run(xin, lab, md, True)
        torch.cuda.current_stream(self.device).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._run(xin, lab, md, True)
        self._graphs[n] = g
        return self
