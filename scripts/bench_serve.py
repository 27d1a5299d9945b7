#!/usr/bin/env python3
"""Serving throughput / latency of ClusterPredictor on one GPU.

    python scripts/bench_serve.py [--d 128 --k 1024 --dtype bf16]

For each batch size: eager requests (fp32 rows -> layout copy + assignment kernel) and
hipGraph replays of the same request; device time per request from HIP events (median
of --reps), rows/s = batch / time.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--batches", default="1024,16384,262144,4194304")
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    import torch
    from tensorflow_distributed_clustering_amd.serving import ClusterPredictor
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    c = torch.randn(a.k, a.d, generator=g, device=dev)
    p = ClusterPredictor(c, dtype=a.dtype, device=dev)
    for b in [int(v) for v in a.batches.split(",")]:
        x = torch.randn(b, a.d, generator=g, device=dev)
        out = {"batch": b, "d": a.d, "k": a.k, "dtype": a.dtype, "backend": p.backend}
        for mode in ("eager", "graph"):
            if mode == "graph":
                p.capture(b)
            for _ in range(3):
                p.predict(x, copy=False)
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                p.predict(x, copy=False)
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            ts.sort()
            ms = ts[len(ts) // 2]
            out[f"{mode}_us"] = ms * 1e3
            out[f"{mode}_rows_per_s"] = b / (ms * 1e-3)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
