#!/usr/bin/env python3
"""Larger-than-HBM clustering from an NPZ file: the completed version of the
reference's `notebooks/batching_tests.ipynb`. That notebook's tf.data streaming hung in
TF_ExtendGraph (`:332-348`).

The NPZ member `X` is memory-mapped (no pickle). Each rank takes its `array_split`
shard. The HBM planner keeps what fits resident and streams the rest through the
native RowStreamer: pinned ring, H2D on a copy stream. Every pass is the exact Lloyd
step, with one all-reduce per pass.

    python examples/out_of_core_npz.py --data class-data.npz --k 1024 --hbm_budget_gb 64
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", required=True)
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--hbm_budget_gb", type=float, default=0.0)
    ap.add_argument("--chunk_rows", type=int, default=0)
    a = ap.parse_args(argv)
    import tensorflow_distributed_clustering_amd as tdc
    from tensorflow_distributed_clustering_amd.data.npz import load_shard, open_npz_member

    comm = tdc.init_comm()
    xmm = open_npz_member(a.data, "X")  # memory map: the shard is not copied here
    n = xmm.shape[0]
    s, e = comm.shard(n)
    cfg = tdc.ClusterConfig(n_clusters=a.k, max_iter=a.iters, dtype=a.dtype,
                            hbm_budget_gb=a.hbm_budget_gb, chunk_rows=a.chunk_rows)
    r = tdc.KMeans(cfg, comm).fit(xmm[s:e], n_global=n, row_offset=s).result_
    if comm.is_root:
        print(json.dumps({"n": n, "streamed": r.streamed, "n_iter": r.n_iter,
                          "points_per_sec": r.points_per_sec, "inertia": r.inertia,
                          "backend": r.backend}))
    tdc.parallel.dist.destroy_comm()


if __name__ == "__main__":
    main()
