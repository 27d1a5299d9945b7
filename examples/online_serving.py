#!/usr/bin/env python3
"""Online clustering + serving: fit on a first batch, keep the centres current with
``MiniBatchKMeans.partial_fit`` as new batches arrive, and answer assignment requests
with a ``ClusterPredictor`` (prepared centroid operands; on a GPU the bf16 MFMA kernel,
optionally replayed from a hipGraph per request size).

The reference only clusters a fixed dataset and labels the points it was fitted on
(`scripts/distribuitedClustering.py:255,282`); this is the deployment-side workflow.

    python examples/online_serving.py [--d 64 --k 32 --batches 20 --batch 8192]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--d", type=int, default=64)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--batches", type=int, default=20)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--requests", type=int, default=20)
    ap.add_argument("--request_rows", type=int, default=1024)
    a = ap.parse_args()
    import torch
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
    from tensorflow_distributed_clustering_amd.ops import reference as ref

    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    dtype = "bf16" if dev.type == "cuda" else "fp32"
    stream = gaussian_blobs(a.batches * a.batch, a.d, a.k, seed=7, device=dev)
    mb = tdc.MiniBatchKMeans(tdc.ClusterConfig(n_clusters=a.k, dtype=dtype, init="kmeans++",
                                               seed=1), device=dev)
    for b in range(a.batches):  # data arrives in batches
        mb.partial_fit(stream[b * a.batch:(b + 1) * a.batch])
    centers = mb.cluster_centers_
    pred = tdc.ClusterPredictor(centers, dtype=dtype, device=dev)
    if dev.type == "cuda":
        pred.capture(a.request_rows)
    reqs = gaussian_blobs(a.requests * a.request_rows, a.d, a.k, seed=8, row_offset=10**7,
                          device=dev)
    lat = []
    agree = 0.0
    for r in range(a.requests):
        q = reqs[r * a.request_rows:(r + 1) * a.request_rows]
        t0 = time.perf_counter()
        lab = pred.predict(q)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        lat.append((time.perf_counter() - t0) * 1e6)
        want, _ = ref.assign(q.double(), torch.as_tensor(centers, device=dev), exact=True)
        agree += (lab.long() == want.long()).float().mean().item() / a.requests
    lat.sort()
    print(json.dumps({"device": str(dev), "backend": pred.backend, "k": a.k, "d": a.d,
                      "batches_seen": mb.engine_.n_iter, "label_agreement": agree,
                      "request_rows": a.request_rows, "p50_us": lat[len(lat) // 2],
                      "p99_us": lat[min(len(lat) - 1, int(0.99 * len(lat)))]}))


if __name__ == "__main__":
    main()
