"""Phase timers with explicit device synchronisation.

The reference timed ``sess.run`` calls with ``time.time()`` (C18,
`scripts/distribuitedClustering.py:150-166,265-280`); ``sess.run`` is synchronous, so
its numbers include the device work.  A PyTorch/HIP launch is asynchronous, so every
timer here brackets its region with a device synchronize (and a process-group barrier
where the caller asks for one) to keep the phase definitions comparable.
"""
from __future__ import annotations

import contextlib
import time
from contextlib import contextmanager

import torch


def sync(device) -> None:
    device = torch.device(device)
    if device.type == "cuda":
        torch.cuda.synchronize(device)


class DeviceTimer:
    """Wall-clock timer synchronised with the device at start and stop."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.t0 = None

    def start(self):
        sync(self.device)
        self.t0 = time.perf_counter()

    def stop(self) -> float:
        sync(self.device)
        return time.perf_counter() - self.t0


@contextmanager
def phase(device, out: dict, name: str):
    sync(device)
    t0 = time.perf_counter()
    try:
        yield
    finally:
        sync(device)
        out[name] = out.get(name, 0.0) + (time.perf_counter() - t0)


@contextlib.contextmanager
def profiled(out_dir: str, rank: int = 0):
    """torch.profiler around a block (CPU + ROCm activities via roctracer): writes
    ``trace_rank<r>.json`` (chrome://tracing) and ``kernels_rank<r>.txt`` to out_dir."""
    import os
    from torch.profiler import ProfilerActivity, profile
    os.makedirs(out_dir, exist_ok=True)
    acts = [ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(ProfilerActivity.CUDA)
    with profile(activities=acts, record_shapes=False) as prof:
        yield prof
    prof.export_chrome_trace(os.path.join(out_dir, f"trace_rank{rank}.json"))
    key = "cuda_time_total" if torch.cuda.is_available() else "cpu_time_total"
    with open(os.path.join(out_dir, f"kernels_rank{rank}.txt"), "w") as f:
        f.write(prof.key_averages().table(sort_by=key, row_limit=40))
