#!/usr/bin/env python3
"""The reference notebook `notebooks/visualization.ipynb`.

The notebook ran a K-Means variant whose per-GPU update is
`unsorted_segment_sum(X, labels, K)` with a NaN -> 0 guard (`:256-271`). Here that is
`empty_cluster="zero"`, and the N2 kernels are the segment sum. The notebook also ran
FCM with an explicit fuzzifier (`:83-175`; its `M=2` was shadowed by the data
dimension). Here the fuzzifier is the `fuzzifier` field and takes effect. Every run
reports its inertia cost, which the notebook had commented out "for performance"
(`:273-275`). Both runs write 2-D scatter plots (`:189-199,336-346`).

    python examples/segment_sum_variant.py --n 200000 --k 5
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200_000)
    ap.add_argument("--k", type=int, default=5)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--plot_prefix", default="visualization")
    a = ap.parse_args(argv)
    import torch
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.data.synth import gaussian_blobs
    from tensorflow_distributed_clustering_amd.utils.plots import scatter_svg

    dev = "cuda" if torch.cuda.is_available() else "cpu"
    x = gaussian_blobs(a.n, 2, a.k, seed=7, dtype=torch.float64, device=dev)
    km = tdc.KMeans(tdc.ClusterConfig(n_clusters=a.k, max_iter=a.iters, dtype="fp64",
                                      init="random", empty_cluster="zero", seed=1)).fit(x).result_
    fcm = tdc.FuzzyCMeans(tdc.ClusterConfig(n_clusters=a.k, max_iter=a.iters, dtype="fp64",
                                            init="random", fuzzifier=2.0, seed=1)).fit(x).result_
    for name, r in (("kmeans_segment_sum", km), ("fcm_m2", fcm)):
        scatter_svg(f"{a.plot_prefix}_{name}.svg", x[:10000].cpu().numpy(),
                    r.labels[:10000].cpu().numpy(), r.init_centers, r.centers, title=name)
    print(json.dumps({"kmeans_inertia": km.inertia, "kmeans_n_iter": km.n_iter,
                      "fcm_centers": fcm.centers.tolist()}))


if __name__ == "__main__":
    main()
