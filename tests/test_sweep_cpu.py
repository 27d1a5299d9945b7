"""Sweep driver + profiler-log compiler (reference scripts/new_experiment.py, compileResults.py)."""
import csv
import os
import subprocess
import sys

import pytest

from tensorflow_distributed_clustering_amd import sweep
from tensorflow_distributed_clustering_amd.utils import profparse as pp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

NVPROF_LOG = """==1234== NVPROF is profiling process 1234, command: python distribuitedClustering.py
==1234== Profiling application: python distribuitedClustering.py
==1234== Profiling result:
            Type  Time(%)      Time     Calls       Avg       Min       Max  Name
 GPU activities:   61.50%  1.2300ms        20  61.500us  60.000us  70.000us  void tensorflow::BiasNCHWKernel<double>(int, double const *)
                   38.50%  770.00us        40  19.250us  1.0000us  40.000us  [CUDA memcpy HtoD]
      API calls:   90.00%  2.50000s        10  250.00ms  1.0000ms  1.00000s  cudaMalloc
                   10.00%  277.78ms         5  55.556ms  100.00ns  277.00ms  cuInit
"""


def test_time_units():
    assert pp.time_to_seconds("1.5ms") == pytest.approx(1.5e-3)
    assert pp.time_to_seconds("250ns") == pytest.approx(2.5e-7)
    assert pp.time_to_seconds("2.0s") == 2.0
    assert pp.time_to_seconds("1.5m") == 90.0
    with pytest.raises(ValueError):
        pp.time_to_seconds("abc")


def test_config_name_roundtrip():
    n = pp.config_name("distributedKMeans", 8, 25_000_000, 5, 3)
    assert n == "distributedKMeans-GPUs8-n_obs25000000-n_dims5-K3"
    assert pp.parse_config_name(n + ".log") == {"method": "distributedKMeans", "n_GPUs": 8,
                                                "n_obs": 25_000_000, "n_dim": 5, "K": 3}
    assert pp.parse_config_name("random.log") is None


def test_nvprof_parse():
    prof, api = pp.parse_nvprof_text(NVPROF_LOG)
    assert len(prof) == 2 and len(api) == 2
    assert prof[0]["NumCalls"] == 20 and prof[0]["Time"] == pytest.approx(1.23e-3)
    assert prof[1]["CallName"] == "[CUDA memcpy HtoD]"
    assert api[0]["CallName"] == "cudaMalloc" and api[0]["MaxCallTime"] == pytest.approx(1.0)


def _rocprof_dir(path):
    os.makedirs(path)
    with open(os.path.join(path, "run_kernel_stats.csv"), "w") as f:
        f.write('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"\n')
        f.write('"tdc::assign_mfma_bf16_ring_kernel<128, 2>",20,50000000,2500000.0,76.9,2400000,2600000,1.0\n')
        f.write('"tdc::segsum_kernel<bf16>",20,15000000,750000.0,23.1,700000,800000,1.0\n')


def test_compile_results_cli(tmp_path):
    inp = tmp_path / "logs"
    inp.mkdir()
    (inp / "distributedFuzzyCMeans-GPUs2-n_obs1000-n_dims5-K3.log").write_text(NVPROF_LOG)
    _rocprof_dir(str(inp / "distributedKMeans-GPUs1-n_obs1000-n_dims5-K3"))
    (inp / "notes.txt").write_text("ignored")
    out = tmp_path / "out"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "compileResults.py"),
                        "--input_dir", str(inp), "--output_dir", str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    kfile = out / "profling_result_distributedKMeans-GPUs1-n_obs1000-n_dims5-K3.csv"
    rows = list(csv.reader(open(kfile)))
    assert rows[0] == [""] + pp.COLUMNS
    assert rows[1][7].startswith("tdc::assign") and float(rows[1][2]) == pytest.approx(0.05)
    assert (out / "API_calls_distributedFuzzyCMeans-GPUs2-n_obs1000-n_dims5-K3.csv").exists()
    summ = list(csv.DictReader(open(out / "summary.csv")))
    assert {s["method"] for s in summ} == {"distributedKMeans", "distributedFuzzyCMeans"}


def test_sweep_plan_matches_reference_grid():
    g = sweep.GRIDS["reference"]
    runs = sweep.plan(g["n_obs"], g["n_dims"], g["K"], g["gpus"], g["methods"])
    assert len(runs) == 320  # = rows of scripts/executions_log.csv
    assert runs[0].name == "distributedKMeans-GPUs1-n_obs100000000-n_dims5-K15"
    g = sweep.GRIDS["legacy"]
    assert len(sweep.plan(g["n_obs"], g["n_dims"], g["K"], g["gpus"], g["methods"])) == 448


def test_sweep_runs_cli_on_cpu(tmp_path):
    log = tmp_path / "exec.csv"
    data = tmp_path / "d.npz"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "new_experiment.py"),
                        "--n_obs", "3000", "--K", "3", "--gpus", "1", "--profiler", "none",
                        "--n_max_iters", "5", "--log_file", str(log), "--data_file", str(data),
                        "--data_kind", "blobs", "--timeout", "300", "--", "--device=cpu"],
                       capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Return code: 0" in r.stdout
    rows = list(csv.reader(open(log)))
    assert len(rows) == 3 and rows[0][0] == "method_name"
    assert {rows[1][0], rows[2][0]} == {"distributedKMeans", "distributedFuzzyCMeans"}
    assert all(float(r[rows[0].index("computation_time")]) > 0 for r in rows[1:])


def test_sweep_skip_done(tmp_path):
    log = tmp_path / "exec.csv"
    log.write_text("method_name,seed,num_GPUs,K,n_obs,n_dim,setup_time,initialization_time,"
                   "computation_time,n_iter\n"
                   "distributedKMeans,1,1,3,1000,5,0.1,0.1,0.5,20\n"
                   "distributedFuzzyCMeans,1,1,3,1000,5,InternalError,InternalError,InternalError,20\n")
    assert sweep.completed_runs(str(log)) == {("distributedKMeans", 1, 3, 1000, 5)}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "new_experiment.py"),
                        "--n_obs", "1000", "--K", "3", "--gpus", "1", "--dry_run", "--skip_done",
                        "--log_file", str(log)], capture_output=True, text=True, timeout=120)
    assert "distributedFuzzyCMeans" in r.stdout and "method_name=distributedKMeans" not in r.stdout
