"""Benchmark sweep driver (reference `scripts/new_experiment.py`, `scripts/generate-logs.py`).

The reference regenerated ``class-data.npz`` (sklearn make_classification, D=5, seed
1826273) for each N, then ran every (K, #GPUs, method) under ``nvprof --log-file`` as a
child process and appended one row per run to ``executions_log.csv``
(`scripts/new_experiment.py:30-66`).  Here the same grid runs the MI355X CLI
(`scripts/distribuitedClustering.py`, torchrun-launched one process per GPU) under
``rocprofv3 --kernel-trace --stats``; ``compileResults.py`` consumes the output dirs.

Grids:
  * ``reference`` -- N in {100M,75M,50M,25M}, D=5, K in {15,12,9,6,3}, GPUs 1..8,
    {distributedKMeans, distributedFuzzyCMeans}   (`scripts/new_experiment.py:34-50`)
  * ``legacy``    -- same N/D, K in 2..15, GPUs {8,6,4,2}   (`scripts/generate-logs.py:30-44`;
    the reference script crashed on a 4-vs-5-argument ``make_data`` call at `:38`)
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import time
from dataclasses import dataclass
from typing import List, Optional, Sequence

from .utils.profparse import config_name

GRIDS = {
    "reference": dict(n_obs=[100_000_000, 75_000_000, 50_000_000, 25_000_000], n_dims=[5],
                      K=[15, 12, 9, 6, 3], gpus=[1, 2, 3, 4, 5, 6, 7, 8],
                      methods=["distributedKMeans", "distributedFuzzyCMeans"]),
    "legacy": dict(n_obs=[100_000_000, 75_000_000, 50_000_000, 25_000_000], n_dims=[5],
                   K=list(range(2, 16)), gpus=[8, 6, 4, 2],
                   methods=["distributedKMeans", "distributedFuzzyCMeans"]),
}
DATA_SEED = 1826273
RUN_SEED = 123128

HERE = os.path.dirname(os.path.abspath(__file__))
CLI = os.path.join(os.path.dirname(HERE), "scripts", "distribuitedClustering.py")


@dataclass
class Run:
    method: str
    n_gpus: int
    n_obs: int
    n_dim: int
    k: int

    @property
    def name(self) -> str:
        return config_name(self.method, self.n_gpus, self.n_obs, self.n_dim, self.k)


def plan(n_obs: Sequence[int], n_dims: Sequence[int], ks: Sequence[int], gpus: Sequence[int],
         methods: Sequence[str]) -> List[Run]:
    """Runs in the reference's loop order: N, D, K, GPUs, method."""
    return [Run(m, g, n, d, k) for n in n_obs for d in n_dims for k in ks for g in gpus
            for m in methods]


def command(run: Run, args) -> List[str]:
    cli = [sys.executable, CLI, f"--n_obs={run.n_obs}", f"--n_dim={run.n_dim}", f"--K={run.k}",
           f"--n_GPUs={run.n_gpus}", f"--n_max_iters={args.n_max_iters}", f"--seed={args.seed}",
           f"--log_file={args.log_file}", f"--method_name={run.method}",
           f"--data_file={args.data_file}"] + list(args.cli_extra)
    if args.profiler == "rocprofv3":
        out = os.path.join(args.log_dir, run.name)
        # the program itself follows "--" (no shell/env hop: the profiler's preload must
        # see the python process directly)
        # csv output: *_kernel_stats.csv per run (compileResults.py input), not a rocpd db
        return ["rocprofv3", "--kernel-trace", "--stats", "-f", "csv", "-d", out, "-o", "run",
                "--"] + cli
    return cli


def completed_runs(log_file: str) -> set:
    """(method, GPUs, K, n_obs, n_dim) of rows with a numeric computation_time: the
    sweep-level resume (the reference always re-ran every config)."""
    import csv
    done = set()
    if not os.path.exists(log_file):
        return done
    with open(log_file, newline="") as f:
        for row in csv.DictReader(f):
            try:
                float(row["computation_time"])
            except (KeyError, TypeError, ValueError):
                continue
            done.add((row["method_name"], int(row["num_GPUs"]), int(row["K"]),
                      int(row["n_obs"]), int(row["n_dim"])))
    return done


def make_dataset(path: str, n_obs: int, n_dim: int, seed: int, kind: str) -> None:
    from .data.synth import make_data
    make_data(path, n_obs, n_dim, seed, kind=kind)


def build_parser(default_grid: str = "reference") -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="Distributed clustering benchmark sweep")
    ap.add_argument("--grid", default=default_grid, choices=sorted(GRIDS))
    ap.add_argument("--n_obs", type=int, nargs="+")
    ap.add_argument("--n_dims", type=int, nargs="+")
    ap.add_argument("--K", type=int, nargs="+")
    ap.add_argument("--gpus", type=int, nargs="+")
    ap.add_argument("--methods", nargs="+")
    ap.add_argument("--n_max_iters", type=int, default=20)
    ap.add_argument("--seed", type=int, default=RUN_SEED)
    ap.add_argument("--data_seed", type=int, default=DATA_SEED)
    ap.add_argument("--data_file", default="class-data.npz")
    ap.add_argument("--data_kind", default="classification", choices=["classification", "blobs"])
    ap.add_argument("--log_file", default="executions_log.csv")
    ap.add_argument("--log_dir", default="rocprof_logs")
    ap.add_argument("--profiler", default="rocprofv3", choices=["rocprofv3", "none"])
    ap.add_argument("--skip_unavailable", action="store_true",
                    help="skip GPU counts above what this node has (the CLI would reject them)")
    ap.add_argument("--dry_run", action="store_true", help="print the commands only")
    ap.add_argument("--skip_done", action="store_true",
                    help="skip configs that already have a successful row in --log_file")
    ap.add_argument("--timeout", type=float, default=0, help="per-run timeout in seconds")
    ap.add_argument("cli_extra", nargs="*", help="extra flags for the CLI (after --)")
    return ap


def main(argv: Optional[Sequence[str]] = None, default_grid: str = "reference") -> int:
    args = build_parser(default_grid).parse_args(argv)
    g = GRIDS[args.grid]
    runs = plan(args.n_obs or g["n_obs"], args.n_dims or g["n_dims"], args.K or g["K"],
                args.gpus or g["gpus"], args.methods or g["methods"])
    if args.skip_unavailable:
        import torch
        avail = torch.cuda.device_count() or 1
        runs = [r for r in runs if r.n_gpus <= avail]
    if args.skip_done:
        done = completed_runs(args.log_file)
        runs = [r for r in runs if (r.method, r.n_gpus, r.k, r.n_obs, r.n_dim) not in done]
    t0 = time.time()
    current_data = None
    worst = 0
    if args.profiler == "rocprofv3" and not args.dry_run:
        os.makedirs(args.log_dir, exist_ok=True)
    for r in runs:
        if (r.n_obs, r.n_dim) != current_data:
            if args.dry_run:
                print(f"# make_data({args.data_file}, {r.n_obs}, {r.n_dim}, {args.data_seed})")
            else:
                make_dataset(args.data_file, r.n_obs, r.n_dim, args.data_seed, args.data_kind)
            current_data = (r.n_obs, r.n_dim)
        cmd = command(r, args)
        if args.dry_run:
            print(" ".join(cmd))
            continue
        try:
            rc = subprocess.call(cmd, timeout=args.timeout or None)
        except subprocess.TimeoutExpired:
            rc = 124
        worst = max(worst, rc)
        print(f"{r.name} - Return code: {rc}", flush=True)
    print(f"total wall time {time.time() - t0:.1f} s")
    return 0 if worst in (0, 1) else worst
