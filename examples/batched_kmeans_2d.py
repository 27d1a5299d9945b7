#!/usr/bin/env python3
"""The reference notebook `notebooks/New-Distributed-KMeans.ipynb` end to end.

The notebook clustered 500M 2-D points on 8 GPUs. It split the data into size-planned
batches (`:190-207`), clustered every batch independently and averaged the centers
(`:225-468`). Then it scatter-plotted the first 10k points with the initial and final
centers (`:502-555`).

Here the whole shard stays resident on each GPU: 500M x 2 fp64 is 8 GB, a small part of
288 GB. One exact distributed Lloyd / FCM run replaces the batch averaging. Run one
process per GPU:

    python examples/batched_kmeans_2d.py --n 500000000 --k 4          # 1 GPU (or CPU)
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/batched_kmeans_2d.py
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=500_000_000)
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--dtype", default="fp64")
    ap.add_argument("--plot_prefix", default="batched_2d")
    a = ap.parse_args(argv)
    import torch
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
    from tensorflow_distributed_clustering_amd.utils.plots import scatter_svg

    comm = tdc.init_comm()
    s, e = comm.shard(a.n)
    x = gaussian_blobs(e - s, 2, a.k, seed=1, row_offset=s, dtype=torch.float64, device=comm.device)
    out = {}
    for name, model in (("kmeans", tdc.KMeans), ("fcm", tdc.FuzzyCMeans)):
        cfg = tdc.ClusterConfig(n_clusters=a.k, max_iter=a.iters, dtype=a.dtype, init="random",
                                seed=3, fuzzifier=2.0)
        r = model(cfg, comm).fit(x, n_global=a.n, row_offset=s).result_
        out[name] = {"computation_time": r.computation_time, "n_iter": r.n_iter,
                     "points_per_sec": r.points_per_sec, "backend": r.backend}
        if comm.is_root:
            scatter_svg(f"{a.plot_prefix}_{name}.svg", x[:10000].cpu().numpy(),
                        r.labels[:10000].cpu().numpy(), r.init_centers, r.centers,
                        title=f"{name} N={a.n} K={a.k}")
    if comm.is_root:
        print(json.dumps(out))
    tdc.parallel.dist.destroy_comm()


if __name__ == "__main__":
    main()
