#!/usr/bin/env python3
"""Micro-benchmark of the wide-D / fp8 assignment kernel (csrc/assign_bigd.hip).

    python scripts/bench_bigd.py --n 5000000 --d 768 --k 65536 --dtype fp8 [--kg-bytes B]
Prints ms per call and effective dense PF/s (2*N*K*D flops).
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=5_000_000)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--k", type=int, default=65536)
    ap.add_argument("--dtype", default="fp8", choices=["fp8", "bf16"])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--kg-tiles", type=int, default=-1, help="-1: library default")
    a = ap.parse_args()
    import torch
    from tensorflow_distributed_clustering_amd import _native
    from tensorflow_distributed_clustering_amd.ops import fp8_dim, kgroup_tiles, wide_bf16_dim
    from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
    ops = _native.require()
    dev = torch.device("cuda", 0)
    x = gaussian_blobs(a.n, a.d, 256, seed=1, dtype=torch.bfloat16, device=dev)
    c = x[torch.randperm(a.n, device=dev)[: a.k]].float().contiguous()
    kp = (a.k + 31) // 32 * 32
    labels = torch.empty(a.n, dtype=torch.int32, device=dev)
    keys = torch.full((a.n,), -1, dtype=torch.int64, device=dev)
    if a.dtype == "fp8":
        dp = fp8_dim(a.d)
        x8 = torch.empty(a.n, dp, dtype=torch.float8_e4m3fn, device=dev)
        xs = torch.empty(a.n, dp // 32, dtype=torch.uint8, device=dev)
        xn = torch.empty(a.n, dtype=torch.float32, device=dev)
        ops.quant_fp8(x, a.n, 0, x8, xs, xn)
        cm = torch.empty(kp, dp, dtype=torch.float8_e4m3fn, device=dev)
        cs = torch.empty(kp, dp // 32, dtype=torch.uint8, device=dev)
        cn = torch.empty(kp, dtype=torch.float32, device=dev)
        ops.quant_fp8(c, a.k, 1, cm, cs, cn)
        kg = kgroup_tiles(dp + dp // 32 + 4, kp) if a.kg_tiles < 0 else a.kg_tiles
        call = lambda: ops.assign_bigd(x8, xs, xn, cm, cs, cn, kg, labels, None, keys)
    else:
        dp = wide_bf16_dim(a.d)
        xb = torch.zeros(a.n, dp, dtype=torch.bfloat16, device=dev)
        xb[:, : a.d] = x
        xn = xb.float().pow(2).sum(1)
        cm = torch.zeros(kp, dp, dtype=torch.bfloat16, device=dev)
        cn = torch.zeros(kp, dtype=torch.float32, device=dev)
        ops.finalize(None, None, c, 0, None, cm, cn)
        kg = kgroup_tiles(dp * 2 + 4, kp) if a.kg_tiles < 0 else a.kg_tiles
        call = lambda: ops.assign_bigd(xb, None, xn, cm, None, cn, kg, labels, None, keys)
    call()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        call()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.reps * 1e3
    fl = 2.0 * a.n * a.k * dp
    print(f"assign_bigd {a.dtype} N={a.n} D={a.d}(DP={dp}) K={a.k} kg={kg}: {ms:.3f} ms  "
          f"{fl / ms / 1e12:.3f} PF/s", flush=True)


if __name__ == "__main__":
    main()
