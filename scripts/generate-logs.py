#!/usr/bin/env python3
"""Older sweep grid (reference `scripts/generate-logs.py`): K in 2..15, GPUs {8,6,4,2}.

The reference version crashed before its first run (4-argument call of a 5-argument
``make_data``, `scripts/generate-logs.py:7,38`); this one runs the intended grid through
the same driver as ``new_experiment.py``.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tensorflow_distributed_clustering_amd.sweep import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(default_grid="legacy"))
