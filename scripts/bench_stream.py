#!/usr/bin/env python3
"""Host-streamed data path throughput: native RowStreamer (f32/f64 -> bf16/fp32, worker
threads) -> pinned ring -> H2D on a copy stream -> consumer.

    python scripts/bench_stream.py --n 20000000 --d 128 [--src f32|f64] [--dst bf16|fp32]
Prints host->device GB/s of source bytes for a pass that only touches each chunk, and
one streamed Lloyd iteration vs the resident one.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20_000_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--src", default="f32", choices=["f32", "f64"])
    ap.add_argument("--dst", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--chunk", type=int, default=1 << 21)
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    import numpy as np
    import torch
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.data.stream import HostSource
    from tensorflow_distributed_clustering_amd.ops import padded_dim
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    x = rng.standard_normal((a.n, a.d), dtype=np.float32)
    if a.src == "f64":
        x = x.astype(np.float64)
    width = padded_dim(a.d) if a.dst == "bf16" else a.d
    layout = (torch.bfloat16 if a.dst == "bf16" else torch.float32, width)
    hs = HostSource(x, layout, dev, n_pinned=3, n_threads=a.threads)
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        acc = torch.zeros((), device=dev)
        for _, c in hs.chunks(a.chunk):
            acc += c[0, 0].float()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    print(f"stream pass: {x.nbytes / dt / 1e9:.2f} GB/s of {a.src} source "
          f"({a.n * width * (2 if a.dst == 'bf16' else 4) / dt / 1e9:.2f} GB/s H2D), {dt*1e3:.1f} ms",
          flush=True)
    cfg = tdc.ClusterConfig(n_clusters=a.k, max_iter=3, dtype=a.dst, init="random",
                            chunk_rows=a.chunk, label_pass=False)
    r = tdc.KMeans(cfg, device=dev).fit(x).result_
    print(f"streamed Lloyd: {r.computation_time / r.n_iter * 1e3:.1f} ms/iter "
          f"({r.points_per_sec / 1e9:.2f} G points/s)", flush=True)
    xr = torch.from_numpy(x).to(dev)
    r2 = tdc.KMeans(cfg.replace(chunk_rows=0), device=dev).fit(xr).result_
    print(f"resident Lloyd: {r2.computation_time / r2.n_iter * 1e3:.1f} ms/iter "
          f"({r2.points_per_sec / 1e9:.2f} G points/s)", flush=True)


if __name__ == "__main__":
    main()
