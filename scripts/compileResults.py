#!/usr/bin/env python3
"""Compile sweep profiler logs into per-configuration CSVs.

Same command line and outputs as the reference (`scripts/compileResults.py:153-175`):

    python compileResults.py --input_dir rocprof_logs/ --output_dir compiled/

For every ``<method>-GPUs<g>-n_obs<n>-n_dims<d>-K<k>`` entry of ``--input_dir`` -- a
rocprofv3 output directory (what ``new_experiment.py`` writes on MI355X) or a legacy
nvprof ``.log`` text file -- writes ``profling_result_<name>.csv`` (GPU kernels) and
``API_calls_<name>.csv`` with columns TimePerc, Time, NumCalls, AvgCallTime, MinCallTime,
MaxCallTime, CallName (seconds).  Additionally writes ``summary.csv`` (one row per config).
"""
import argparse
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tensorflow_distributed_clustering_amd.utils.profparse import compile_entry, summarize  # noqa: E402


def is_valid_dir(parser, arg):
    if not os.path.exists(arg):
        parser.error("The directory %s does not exist!" % arg)
    return arg


def main(input_dir: str, output_dir: str) -> int:
    os.makedirs(output_dir, exist_ok=True)
    for i, entry in enumerate(sorted(os.listdir(input_dir)), 1):
        print(i, "- input_file_name = ", entry)
        compile_entry(os.path.join(input_dir, entry), output_dir)
    rows = summarize(input_dir)
    if rows:
        with open(os.path.join(output_dir, "summary.csv"), "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0]))
            w.writeheader()
            w.writerows(rows)
    return 1


if __name__ == "__main__":
    parser = argparse.ArgumentParser(description="Compile Distributed K-Means profiler results.")
    parser.add_argument("--input_dir", dest="input_dir", required=True, metavar="DIR",
                        type=lambda x: is_valid_dir(parser, x),
                        help="The directory where profiler logs are located")
    parser.add_argument("--output_dir", dest="output_dir", required=True, metavar="DIR",
                        help="The directory where compiled CSVs will be saved (created)")
    args = parser.parse_args()
    main(args.input_dir, args.output_dir)
