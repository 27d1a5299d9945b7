"""Flag-compatible command line of the reference engine.

    python scripts/distribuitedClustering.py --n_obs N --n_dim D --K K --n_GPUs G \\
        --n_max_iters I --seed S --log_file out.csv --method_name distributedKMeans \\
        --data_file data.npz [extensions...]

Reference: `scripts/distribuitedClustering.py:411-491`.  Compatible surface:
* the nine required flags, same spellings (``--n_GPUs``), same validators / errors
  (`:18-70`): integer parse, data file must exist, method whitelist, G in 1..available;
* the log CSV: created with the exact 10-column header at argument-parse time
  (`:30-36`), one ``str()``-joined row appended per run (`:379-405`); on an exception the
  class name is written into the three time columns (`:362-374`);
* exit status 1 only when the caught exception is a ``ValueError`` (`:376,491`).

Differences (documented, deliberate): ``--seed`` seeds centroid init; the GPU subset is
``0..G-1`` (one process per GPU via torchrun) instead of a random unseeded pick (`:69`);
OOM falls back to exact streamed Lloyd instead of clustering independent batches and
averaging their centers (`:296-360`).  Extensions: ``--dtype --init --fuzzifier
--empty_cluster --tol --device --backend --centroids_out --labels_out --compat
--checkpoint --resume --extended_log``.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import traceback

LOG_HEADER = ["method_name", "seed", "num_GPUs", "K", "n_obs", "n_dim", "setup_time",
              "initialization_time", "computation_time", "n_iter"]
METHODS = ["distributedKMeans", "distributedFuzzyCMeans"]


# ----------------------------------------------------------------------- validators
def check_file_exists(parser, arg):
    data_file = str(arg)
    if os.path.exists(data_file):
        return data_file
    parser.error("Data File not Found")


def is_valid_file(parser, arg):
    if not os.path.exists(arg):
        with open(arg, "w") as f:
            f.write(",".join(LOG_HEADER) + "\n")
    return str(arg)


def make_valid_int(parser, arg):
    try:
        return int(arg)
    except ValueError:
        parser.error("Invalid Integer")


def make_valid_method(parser, arg):
    method_name = str(arg)
    if method_name in METHODS + ["miniBatchKMeans"]:
        return method_name
    parser.error("Invalid Method Name")


def available_devices(device: str) -> int:
    import torch
    if device == "cpu":
        return os.cpu_count() or 1
    n = torch.cuda.device_count()  # does not initialise the GPU on this image
    if n == 0 and device == "auto":
        return os.cpu_count() or 1
    return n


def make_valid_gpus(parser, arg, device="auto"):
    n = make_valid_int(parser, arg)
    avail = available_devices(device)
    if n > avail:
        parser.error("Number of GPUs Given is More Then Available")
    if n <= 0:
        parser.error("Number of GPUs Given is Non Positive")
    return n


def build_parser():
    parser = argparse.ArgumentParser(description="Compile Distribuited K Means Results.")
    dev_hint = "auto"
    for a in sys.argv:
        if a.startswith("--device="):
            dev_hint = a.split("=", 1)[1]
    if "--device" in sys.argv:
        i = sys.argv.index("--device")
        if i + 1 < len(sys.argv):
            dev_hint = sys.argv[i + 1]
    I = lambda x: make_valid_int(parser, x)
    parser.add_argument("--n_obs", dest="n_obs", required=True, metavar="int", type=I,
                        help="Number of Observations for the Test !!!")
    parser.add_argument("--n_dim", dest="n_dim", required=True, metavar="int", type=I,
                        help="Number of Dimensions for the Test !!!")
    parser.add_argument("--K", dest="K", required=True, metavar="int", type=I,
                        help="Number of K Centers for the Test !!!")
    parser.add_argument("--n_GPUs", dest="n_GPUs", required=True, metavar="int",
                        type=lambda x: make_valid_gpus(parser, x, dev_hint), help="Number of GPUs !!!")
    parser.add_argument("--n_max_iters", dest="n_max_iters", required=True, metavar="int", type=I,
                        help="Number of iterations before stopping!!!")
    parser.add_argument("--seed", dest="seed", required=True, metavar="int", type=I,
                        help="Seed Value !!!")
    parser.add_argument("--log_file", dest="log_file", required=True, metavar="FILE",
                        type=lambda x: is_valid_file(parser, x),
                        help="log_file Name, this would be a CSV !!!")
    parser.add_argument("--method_name", dest="method_name", required=True, metavar="str",
                        type=lambda x: make_valid_method(parser, x),
                        help="Method Name Can Be :distribuitedKMeans or distribuitedFuzzyCMeans !!!")
    parser.add_argument("--data_file", dest="data_file", required=True, metavar="str",
                        type=lambda x: check_file_exists(parser, x),
                        help="Unable to find data file !!!")
    # ---- extensions (all optional) ----
    parser.add_argument("--dtype", default="auto", choices=["auto", "fp64", "fp32", "bf16", "fp8"])
    parser.add_argument("--init", default="kmeans++", choices=["kmeans++", "kmeans||", "first_k", "random"])
    parser.add_argument("--fuzzifier", type=float, default=None,
                        help="FCM m (default: the data dimension, as the reference)")
    parser.add_argument("--empty_cluster", default="keep",
                        choices=["keep", "nan", "nan_any", "zero", "reseed"])
    parser.add_argument("--tol", type=float, default=0.0)
    parser.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"])
    parser.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"])
    parser.add_argument("--batch_size", type=int, default=0, help="miniBatchKMeans rows/rank/step")
    parser.add_argument("--chunk_rows", type=int, default=0, help="stream the shard in chunks")
    parser.add_argument("--centroids_out", default=None)
    parser.add_argument("--labels_out", default=None)
    parser.add_argument("--extended_log", default=None, help="JSON-lines file with derived metrics")
    parser.add_argument("--compat", action="store_true",
                        help="reference bug-compat: NaN empty clusters, first-K init")
    parser.add_argument("--checkpoint", default=None,
                        help="NPZ checkpoint of the centroids (written by rank 0)")
    parser.add_argument("--checkpoint_every", type=int, default=0,
                        help="iterations between checkpoints (0: only at the end)")
    parser.add_argument("--resume", action="store_true",
                        help="continue from --checkpoint if it exists")
    parser.add_argument("--hbm_budget_gb", type=float, default=0.0,
                        help="per-GPU memory budget for the stream planner (0: free HBM)")
    parser.add_argument("--log_device_placement", action="store_true",
                        help="print rank -> device / shard / kernel backend (the reference's "
                             "tf.ConfigProto(log_device_placement=True))")
    parser.add_argument("--plot_out", default=None,
                        help="SVG scatter of the first 10k points of rank 0 with initial and "
                             "final centers")
    parser.add_argument("--log_every", type=int, default=0,
                        help="every N iterations print (and record in --extended_log) the max "
                             "centroid shift and the inertia of that iteration")
    parser.add_argument("--torch_profile", default=None, metavar="DIR",
                        help="record the fit with torch.profiler (ROCm/roctracer) and write a "
                             "chrome trace + kernel table to DIR")
    parser.add_argument("--collective_timeout", type=float, default=600.0,
                        help="seconds before a stuck collective raises (init_process_group)")
    parser.add_argument("--graph", action="store_true",
                        help="replay each iteration from a captured HIP graph (1 GPU)")
    parser.add_argument("--deterministic", action="store_true",
                        help="run-to-run bitwise reproducible centroid update")
    parser.add_argument("--update", default="auto", choices=["auto", "full", "delta"],
                        help="K-Means centroid update: delta moves only the rows whose label "
                             "changed between fp64 running totals (auto: where supported)")
    parser.add_argument("--spherical", action="store_true",
                        help="cosine (spherical) K-Means: unit-normalised rows and centroids")
    parser.add_argument("--dist_debug", action="store_true",
                        help="check every collective for rank mismatches "
                             "(TORCH_DISTRIBUTED_DEBUG=DETAIL)")
    parser.add_argument("--fp8_recheck", type=float, default=0.0,
                        help="fp8: re-check near ties (fp8 margin within this fraction of the "
                             "runner-up distance) exactly in fp32; 0 = off")
    parser.add_argument("--algorithm", default="lloyd", choices=["lloyd", "bounded"],
                        help="bounded: exact Lloyd that re-assigns only the rows its Hamerly "
                             "bounds cannot settle (resident bf16 MFMA path)")
    parser.add_argument("--no_warmup", action="store_true",
                        help="time the first iteration too (the reference's computation_time "
                             "includes its first sess.run); by default one discarded step "
                             "runs before the timer, its first-launch cost counted in setup_time")
    parser.add_argument("--num_batches", type=int, default=1,
                        help="reference batch mode: cluster N array_split batches independently, "
                             "sum the phase times and average the centers (default 1: one "
                             "exact fit over all rows)")
    return parser


def resolve_dtype(dtype: str, k: int, d: int, method: str = "distributedKMeans") -> str:
    """``--dtype auto``: the reference's data is fp64 and its distances are fp64
    (`scripts/distribuitedClustering.py:221-234`).  K-Means keeps fp64 up to D = 1024: the
    fp64 path assigns on the matrix cores (bf16x3 scores) and re-checks every row the error
    bound cannot certify in fp64, so its labels are the fp64 argmin (ops.HipX3Lloyd); past
    D = 1024 it runs fp32 exact tiles.  FCM keeps fp64 up to D = 16 (fused small-K*D
    kernel) and from K = 64 at any D (both GEMM-shaped passes on the fp64 matrix cores,
    ops.fcm_f64_mfma: from D = 64 fp32 data is promoted to the same path, so fp64 costs
    nothing extra; at D = 32 it costs ~1.35x the fp32 tower); in between it runs the exact
    fp32 SIMT tower (~1.6x the fp64 tower's speed).  Nothing is silently dropped to bf16:
    the resolved dtype is printed and written to --extended_log."""
    if dtype != "auto":
        return dtype
    if method == "distributedFuzzyCMeans":
        from .ops import fcm_f64_mfma
        return "fp64" if (d <= 16 or fcm_f64_mfma(k, d, "fp64")) else "fp32"
    return "fp64" if d <= 1024 else "fp32"


def format_row(vals) -> str:
    return ",".join(str(v) for v in vals) + "\n"


def write_centroids_csv(path: str, centers) -> None:
    with open(path, "w") as f:
        for row in centers:
            f.write(",".join(repr(float(v)) for v in row) + "\n")


def write_labels_csv(path: str, labels) -> None:
    import numpy as np
    np.savetxt(path, np.asarray(labels, dtype=np.int64), fmt="%d")


# ----------------------------------------------------------------------------- run
def run(args) -> int:
    import numpy as np
    import torch
    from . import ClusterConfig, FuzzyCMeans, KMeans
    from .data.npz import load_shard
    from .parallel.dist import init_comm

    device = args.device
    if device == "auto":
        device = "cuda" if torch.cuda.device_count() > 0 else "cpu"
    comm = init_comm(device, timeout_s=args.collective_timeout, debug=args.dist_debug)
    status = 0
    result = None
    exc_name = None
    try:
        if args.num_batches > 1:
            from .data.npz import open_npz_member
            x = open_npz_member(args.data_file, "X")  # batches are cut from the global rows
            n_global, row_off = int(x.shape[0]), 0
        else:
            x, n_global, row_off = load_shard(args.data_file, comm.rank, comm.world_size, "X")
        d = x.shape[1]
        if (args.n_obs, args.n_dim) != (n_global, d) and comm.is_root:
            print(f"note: --n_obs/--n_dim are logged only; data file is {n_global}x{d}",
                  file=sys.stderr)
        dtype = resolve_dtype(args.dtype, args.K, d, args.method_name)
        if comm.is_root and args.dtype != dtype:
            print(f"note: --dtype {args.dtype} resolved to {dtype} (D={d}, K={args.K}, "
                  f"{args.method_name}; the reference's fp64 precision where it runs on the "
                  f"matrix cores -- --dtype bf16 trades it for the bf16 MFMA rate)",
                  file=sys.stderr)
        init = "first_k" if args.compat else args.init
        empty = "nan_any" if args.compat else args.empty_cluster
        cfg = ClusterConfig(n_clusters=args.K, max_iter=args.n_max_iters, tol=args.tol,
                            dtype=dtype, init=init, seed=args.seed, fuzzifier=args.fuzzifier,
                            empty_cluster=empty, backend=args.backend,
                            chunk_rows=args.chunk_rows, batch_size=args.batch_size,
                            checkpoint_path=args.checkpoint or "",
                            checkpoint_every=args.checkpoint_every, resume=args.resume,
                            hbm_budget_gb=args.hbm_budget_gb, deterministic=args.deterministic,
                            graph=args.graph, log_every=args.log_every,
                            spherical=args.spherical, algorithm=args.algorithm,
                            fp8_recheck=args.fp8_recheck, warmup=not args.no_warmup,
                            update=args.update)

        def make_model():
            if args.method_name == "distributedKMeans":
                return KMeans(cfg, comm)
            if args.method_name == "distributedFuzzyCMeans":
                return FuzzyCMeans(cfg, comm)
            from .models.minibatch import MiniBatchKMeans
            return MiniBatchKMeans(cfg, comm)

        if args.num_batches > 1:
            from .models.batched import fit_batches_averaged
            result = fit_batches_averaged(make_model, x, n_global, args.num_batches,
                                          comm.rank, comm.world_size)
            x = np.asarray(x[:min(10000, n_global)])  # rows for --plot_out only
        else:
            model = make_model()
            xt = torch.from_numpy(np.asarray(x))
            if args.torch_profile:
                from .utils.timers import profiled
                with profiled(args.torch_profile, comm.rank):
                    model.fit(xt, n_global=n_global, row_offset=row_off)
            else:
                model.fit(xt, n_global=n_global, row_offset=row_off)
            result = model.result_
        if args.log_device_placement:
            name = (torch.cuda.get_device_name(comm.device) if comm.device.type == "cuda"
                    else "host")
            print(f"[placement] rank {comm.rank}/{comm.world_size} local_rank {comm.local_rank} "
                  f"device {comm.device} ({name}) rows [{row_off}, {row_off + x.shape[0]}) "
                  f"backend {result.backend} dtype {dtype}", flush=True)
        if args.plot_out and comm.is_root:
            from .utils.plots import scatter_svg
            scatter_svg(args.plot_out, x, None if result.labels is None else
                        result.labels.cpu().numpy(), result.init_centers, result.centers,
                        title=f"{args.method_name} K={args.K}")
    except Exception:
        exc_type, exc_value, exc_tb = sys.exc_info()
        traceback.print_exc()
        exc_name = exc_type.__name__
        status = 1 if exc_name == "ValueError" else 0

    # phase times: max over ranks (the reference timed the whole multi-GPU step)
    if result is not None:
        setup = comm.max_scalar(result.setup_time)
        init_t = comm.max_scalar(result.initialization_time)
        comp = comm.max_scalar(result.computation_time)
        n_iter = result.n_iter
        labels_all = None
        if args.labels_out and result.labels is not None:
            labels_all = comm.gather_rows_to_root(result.labels)
    if comm.is_root:
        if result is not None:
            vals = [args.method_name, args.seed, comm.world_size, args.K, args.n_obs, args.n_dim,
                    setup, init_t, comp, n_iter]
        else:
            vals = [args.method_name, args.seed, comm.world_size, args.K, args.n_obs, args.n_dim,
                    exc_name, exc_name, exc_name, args.n_max_iters]
        with open(args.log_file, "a") as f:
            f.write(format_row(vals))
        if result is not None:
            if args.centroids_out:
                write_centroids_csv(args.centroids_out, result.centers)
            if args.labels_out and labels_all is not None:
                write_labels_csv(args.labels_out, labels_all.cpu().numpy())
            if args.extended_log:
                with open(args.extended_log, "a") as f:
                    f.write(json.dumps({
                        "method_name": args.method_name, "num_GPUs": comm.world_size,
                        "K": args.K, "n_obs": result.n_global, "n_dim": int(result.centers.shape[1]),
                        "n_iter": n_iter, "computation_time": comp, "backend": result.backend,
                        "dtype": dtype,
                        "points_per_sec": result.n_global * n_iter / comp if comp > 0 else None,
                        "iters_per_sec": n_iter / comp if comp > 0 else None,
                        "warmup_step": not args.no_warmup,
                        "inertia": result.inertia, "history": result.history}) + "\n")
        print("log_file =", args.log_file)
    return status


def _under_launcher() -> bool:
    return "LOCAL_RANK" in os.environ and "WORLD_SIZE" in os.environ


def main(argv=None) -> int:
    if argv is not None:
        sys.argv = [sys.argv[0]] + list(argv)
    parser = build_parser()
    args = parser.parse_args()
    if args.n_GPUs > 1 and not _under_launcher():
        # one process per GPU: re-launch under torchrun as a CHILD (never exec after GPU init)
        import socket
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        target = (["-m", "tensorflow_distributed_clustering_amd.cli"]
                  if os.path.basename(sys.argv[0]) in ("cli.py", "__main__.py") else [sys.argv[0]])
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={args.n_GPUs}", "--master-addr=127.0.0.1",
               f"--master-port={port}"] + target + sys.argv[1:]
        env = dict(os.environ)
        env.setdefault("OMP_NUM_THREADS", "1")
        return subprocess.call(cmd, env=env)
    if _under_launcher() and int(os.environ["WORLD_SIZE"]) != args.n_GPUs:
        parser.error("WORLD_SIZE does not match --n_GPUs")
    try:
        return run(args)
    finally:
        # tear the process group down before interpreter exit: a gloo group left to the
        # exit-time destructors intermittently aborted rank 0 ("terminate called without
        # an active exception") after its outputs were written
        from .parallel.dist import destroy_comm
        destroy_comm()


if __name__ == "__main__":
    sys.exit(main())
