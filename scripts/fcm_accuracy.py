#!/usr/bin/env python3
"""FCM MFMA tower accuracy against the fp64 oracle (ops.reference.fcm_partial, exact
difference form): max |centroid - oracle| / max|oracle centroid|, max relative error of the
weight sums, and label agreement, on the oracle tests' data (points near centroids) and on
Gaussian blobs.

    python scripts/fcm_accuracy.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
    from tensorflow_distributed_clustering_amd.ops import HipMfmaFCM
    from tensorflow_distributed_clustering_amd.ops import reference as ref
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    cases = []
    for n, k, d in [(20001, 1024, 128), (20001, 100, 64)]:
        x = torch.randn(n, d, generator=g, dtype=torch.float64)
        c = x[torch.randperm(n, generator=g)[:k]] + 0.05 * torch.randn(k, d, generator=g,
                                                                       dtype=torch.float64)
        cases.append((f"near n={n} k={k} d={d}", x, c))
    xb = gaussian_blobs(200_000, 128, 1024, seed=3, dtype=torch.float64, device="cpu")
    cb = xb[torch.randperm(xb.shape[0], generator=g)[:1024]] + 0.1
    cases.append(("blobs n=200000 k=1024 d=128", xb, cb))
    for name, x, c in cases:
        for m in (2.0, 3.0):
            xg, cg = x.float().to(dev), c.float().to(dev)
            ops = HipMfmaFCM(xg, c.shape[0], m, True)
            lab = torch.empty(x.shape[0], dtype=torch.int32, device=dev)
            wx = torch.zeros(c.shape[0], x.shape[1], dtype=torch.float64, device=dev)
            ws = torch.zeros(c.shape[0], dtype=torch.float64, device=dev)
            ops.step(cg, lab, wx, ws)
            a, b, lr = ref.fcm_partial(xg.double().cpu(), cg.double().cpu(), m, True, exact=True)
            cen = (wx / ws.clamp_min(1e-300)[:, None]).cpu()
            cref = a / b.clamp_min(1e-300)[:, None]
            ok = b > 1e-12 * b.max()
            ce = float((cen[ok] - cref[ok]).abs().max() / cref[ok].abs().max())
            we = float(((ws.cpu()[ok] - b[ok]).abs() / b[ok]).max())
            ag = float((lab.long().cpu() == lr.long()).double().mean())
            print(f"{name} m={m}: centroid err {ce:.2e} (rel. to max|c|), ws rel err {we:.2e}, "
                  f"label agreement {ag:.5f}")


if __name__ == "__main__":
    main()
