#!/usr/bin/env python3
"""One library GEMM shape, launched back to back, for a PMC pass (scripts/pmc_run.sh): the
MFMA busy fraction hipBLASLt itself reaches on this GPU, to calibrate the fused assign
kernels' busy fractions against (docs/PERF_NOTES.md, round 6).

    python3 scripts/gemm_pmc.py fp8 16384 16384 8192 [reps]
    python3 scripts/gemm_pmc.py bf16 8192 8192 8192 [reps]

Prints the TFLOP/s of the timed reps (the PMC run slows them; quote the timing from an
unprofiled run)."""
import json
import sys
import time

import torch


def main():
    kind, m, n, k = sys.argv[1], *map(int, sys.argv[2:5])
    reps = int(sys.argv[5]) if len(sys.argv) > 5 else 10
    if kind == "fp8":
        a = torch.randn(m, k, device="cuda").to(torch.float8_e4m3fn)
        b = torch.randn(n, k, device="cuda").to(torch.float8_e4m3fn).t()
        one = torch.ones((), device="cuda")
        f = lambda: torch._scaled_mm(a, b, one, one, out_dtype=torch.bfloat16)
    else:
        a = torch.randn(m, k, device="cuda").to(torch.bfloat16)
        b = torch.randn(k, n, device="cuda").to(torch.bfloat16)
        f = lambda: torch.matmul(a, b)
    f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    print(json.dumps({"kind": kind, "shape": [m, n, k], "ms": dt * 1e3,
                      "TFLOP/s": 2.0 * m * n * k / dt / 1e12}), flush=True)


if __name__ == "__main__":
    main()
