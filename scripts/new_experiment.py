#!/usr/bin/env python3
"""Benchmark sweep (reference `scripts/new_experiment.py`): regenerate the dataset per N and
run every (K, #GPUs, method) of the grid under rocprofv3, appending to executions_log.csv.

    python new_experiment.py                          # the reference grid (320 runs)
    python new_experiment.py --n_obs 1000000 --K 3 6 --gpus 1 2 --profiler none
    python new_experiment.py --dry_run                # print the commands
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tensorflow_distributed_clustering_amd.sweep import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
