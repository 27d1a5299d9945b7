#!/usr/bin/env python3
"""Practical bf16 / fp8-class MFMA ceiling on this GPU: hipBLASLt (torch.matmul) on large
square GEMMs with random data, timed back to back.  The fused assign kernels are judged
against this, not only against the ~2.5 PF/s spec (DVFS lowers the clock under dense MFMA
load: MI355X_MICROARCH.md, "DVFS give-back")."""
import json
import time

import torch


def bench(m, n, k, dtype, reps=20):
    a = torch.randn(m, k, device="cuda", dtype=torch.float32).to(dtype)
    b = torch.randn(k, n, device="cuda", dtype=torch.float32).to(dtype)
    for _ in range(3):
        torch.matmul(a, b)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        torch.matmul(a, b)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    return 2.0 * m * n * k / dt / 1e12


def bench_fp8(m, n, k, reps=20):
    """Tensor-wise scaled OCP e4m3 GEMM (torch._scaled_mm -> hipBLASLt)."""
    a = torch.randn(m, k, device="cuda").to(torch.float8_e4m3fn)
    b = torch.randn(n, k, device="cuda").to(torch.float8_e4m3fn).t()  # column-major
    one = torch.ones((), device="cuda")
    f = lambda: torch._scaled_mm(a, b, one, one, out_dtype=torch.bfloat16)
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    return 2.0 * m * n * k / dt / 1e12


out = {}
for (m, n, k) in [(8192, 8192, 8192), (16384, 16384, 8192), (65536, 1024, 128), (131072, 1024, 128)]:
    out[f"bf16 {m}x{n}x{k}"] = round(bench(m, n, k, torch.bfloat16), 1)
# config-5 shaped fp8: a 64K-row point chunk against the 65536 x 768 centroid table
for (m, n, k) in [(8192, 8192, 8192), (16384, 16384, 8192), (65536, 65536, 768)]:
    try:
        out[f"fp8 {m}x{n}x{k}"] = round(bench_fp8(m, n, k), 1)
    except Exception as e:  # pragma: no cover - depends on the hipBLASLt build
        out[f"fp8 {m}x{n}x{k}"] = f"unavailable: {type(e).__name__}: {str(e)[:120]}"
print(json.dumps({"TFLOP/s": out}), flush=True)
