#!/usr/bin/env python3
"""Per-kernel microbenchmarks on one GPU (no data-generation noise; profiler friendly).

    python scripts/bench_kernels.py --n 10000000 --d 128 --k 1024 [--only assign]

Reports device time per call (HIP events, median of --reps) and the derived rates:
assign = 2*N*K*D FLOP (bf16 MFMA), update = bytes of X read.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="", help="comma list of assign,update,update_lds,small,fcm")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--data", default="normal", choices=["normal", "uniform", "blobs"])
    a = ap.parse_args()
    import torch
    from tensorflow_distributed_clustering_amd import _native
    from tensorflow_distributed_clustering_amd.ops import HipBf16Lloyd, NativeUpdate
    ops = _native.require()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    only = set(a.only.split(",")) if a.only else None
    res = {"n": a.n, "d": a.d, "k": a.k}

    def timeit(fn):
        for _ in range(3):
            fn()
        if os.environ.get("KB_WALL"):
            import time
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                fn()
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) * 1e3 / a.reps
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); fn(); e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        return ts[len(ts) // 2]

    if a.data == "normal":
        x = (torch.randn(a.n, a.d, device=dev, generator=g) * 2).to(torch.bfloat16)
        c = torch.randn(a.k, a.d, device=dev, generator=g) * 2
    elif a.data == "uniform":
        x = (torch.rand(a.n, a.d, device=dev, generator=g) * 4 - 2).to(torch.bfloat16)
        c = torch.rand(a.k, a.d, device=dev, generator=g) * 4 - 2
    else:
        from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
        x = gaussian_blobs(a.n, a.d, a.k, seed=0, dtype=torch.bfloat16, device=dev)
        c = x[torch.randperm(a.n, device=dev)[: a.k]].float()
    loc = HipBf16Lloyd(x, a.k)
    loc.prepare(c)
    if os.environ.get("KB_CNORM1"):
        loc.cnorm[: a.k] = 1.0
    labels = torch.zeros(a.n, dtype=torch.int32, device=dev)
    if only is None or "assign" in only:
        ms = timeit(lambda: ops.assign_bf16(loc.x, loc.cm2, loc.cnorm, labels, None))
        res["assign_ms"] = ms
        res["assign_tflops"] = 2.0 * a.n * a.k * loc.dp / ms / 1e9
    if only is not None and "assign_idx" in only:
        # cost of the point loads: the indexed kernel over rows in order, over a 4096-row
        # (1 MiB, L2-resident) window, and over one row (timing only; labels are discarded)
        for name, ri in (("arange", torch.arange(a.n, device=dev, dtype=torch.int32)),
                         ("l2win", torch.arange(a.n, device=dev, dtype=torch.int32) % 4096),
                         ("row0", torch.zeros(a.n, device=dev, dtype=torch.int32))):
            ms = timeit(lambda: ops.assign_bf16_indexed(loc.x, ri, loc.cm2, loc.cnorm, labels,
                                                        None))
            res[f"assign_idx_{name}_ms"] = ms
    ops.assign_bf16(loc.x, loc.cm2, loc.cnorm, labels, None)
    sums =torch.zeros(a.k, a.d, dtype=torch.float32, device=dev)
    counts = torch.zeros(a.k, dtype=torch.float32, device=dev)
    if only is None or "update" in only:
        up = NativeUpdate(ops, a.n, a.k, a.d, torch.bfloat16, dev)
        ms = timeit(lambda: (sums.zero_(), counts.zero_(), up(loc.x, labels, sums, counts)))
        res["update_kind"] = up.kind
        res["update_ms"] = ms
        res["update_GBps"] = a.n * loc.dp * 2 / ms / 1e6
    if only is not None and "update_lds" in only:
        ms = timeit(lambda: (sums.zero_(), counts.zero_(), ops.update(loc.x, labels, sums, counts)))
        res["update_lds_ms"] = ms
    print(json.dumps(res))


if __name__ == "__main__":
    main()
