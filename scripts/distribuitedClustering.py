#!/usr/bin/env python3
"""Flag-compatible entry point of the reference engine
(`scripts/distribuitedClustering.py` in Jhonsonzhangxing/tensorflow-distributed-clustering).

    python scripts/distribuitedClustering.py --n_obs 25000000 --n_dim 5 --K 3 --n_GPUs 8 \
        --n_max_iters 20 --seed 123128 --log_file executions_log.csv \
        --method_name distributedKMeans --data_file class-data.npz

Implementation: tensorflow_distributed_clustering_amd.cli (one process per GPU, RCCL).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tensorflow_distributed_clustering_amd.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
