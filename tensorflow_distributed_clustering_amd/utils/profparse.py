"""Profiler-output parsing for the benchmark sweep (reference `scripts/compileResults.py`).

The reference ran every sweep configuration under ``nvprof --log-file`` and turned each
text log into two CSVs with the columns

    TimePerc, Time, NumCalls, AvgCallTime, MinCallTime, MaxCallTime, CallName

(times in seconds; `scripts/compileResults.py:44-137`).  On MI355X the sweep runs under
``rocprofv3 --kernel-trace --stats`` instead, which writes ``*_kernel_stats.csv`` (GPU
kernels) and, with ``--hip-trace``, ``*_hip_api_stats.csv`` (runtime API calls).  This
module maps both inputs -- rocprofv3 stats directories *and* legacy nvprof text logs --
onto the same column schema, so downstream analysis of either generation of logs is
unchanged.

The configuration is encoded in the log/dir name exactly as the reference sweep named
its logs: ``<method>-GPUs<g>-n_obs<n>-n_dims<d>-K<k>`` (`scripts/new_experiment.py:53`).
"""
from __future__ import annotations

import csv
import glob
import os
import re
from typing import Dict, Iterable, List, Optional, Tuple

COLUMNS = ["TimePerc", "Time", "NumCalls", "AvgCallTime", "MinCallTime", "MaxCallTime", "CallName"]

_UNIT = {"ns": 1e-9, "us": 1e-6, "ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0}
_NAME_RE = re.compile(r"^(?P<method>[A-Za-z]+)-GPUs(?P<gpus>\d+)-n_obs(?P<n_obs>\d+)"
                      r"-n_dims(?P<n_dims>\d+)-K(?P<K>\d+)$")
_NUM_UNIT_RE = re.compile(r"^([-+]?\d*\.?\d+(?:[eE][-+]?\d+)?)([a-zA-Z]*)$")


def time_to_seconds(tok: str) -> float:
    """``'1.234ms'`` -> 0.001234.  A bare number is taken as seconds (nvprof prints units)."""
    m = _NUM_UNIT_RE.match(tok.strip())
    if not m:
        raise ValueError(f"not a time value: {tok!r}")
    val, unit = float(m.group(1)), m.group(2)
    if unit and unit not in _UNIT:
        raise ValueError(f"unknown time unit {unit!r} in {tok!r}")
    return val * _UNIT.get(unit or "s")


def parse_config_name(name: str) -> Optional[Dict[str, object]]:
    """``distributedKMeans-GPUs8-n_obs25000000-n_dims5-K3`` -> config dict (None if no match)."""
    base = os.path.basename(name.rstrip("/"))
    for ext in (".log", ".csv"):
        if base.endswith(ext):
            base = base[: -len(ext)]
    m = _NAME_RE.match(base)
    if not m:
        return None
    d = m.groupdict()
    return {"method": d["method"], "n_GPUs": int(d["gpus"]), "n_obs": int(d["n_obs"]),
            "n_dim": int(d["n_dims"]), "K": int(d["K"])}


def config_name(method: str, n_gpus: int, n_obs: int, n_dim: int, k: int) -> str:
    return f"{method}-GPUs{n_gpus}-n_obs{n_obs}-n_dims{n_dim}-K{k}"


# ----------------------------------------------------------------------------- nvprof
def _nvprof_rows(section: str) -> List[dict]:
    rows = []
    for line in section.splitlines():
        toks = line.split()
        # rows of the summary table start with "<pct>%" possibly after a "GPU activities:"
        # or "API calls:" label
        while toks and not toks[0].endswith("%"):
            toks = toks[1:]
        if len(toks) < 7:
            continue
        try:
            pct = float(toks[0].rstrip("%"))
            row = {"TimePerc": pct, "Time": time_to_seconds(toks[1]), "NumCalls": int(toks[2]),
                   "AvgCallTime": time_to_seconds(toks[3]), "MinCallTime": time_to_seconds(toks[4]),
                   "MaxCallTime": time_to_seconds(toks[5]), "CallName": " ".join(toks[6:])}
        except ValueError:
            continue
        rows.append(row)
    return rows


def parse_nvprof_text(text: str) -> Tuple[List[dict], List[dict]]:
    """(profiling rows, API-call rows) of an nvprof summary log."""
    m = re.search(r"==\d+== Profiling result:", text)
    if not m:
        raise ValueError("no '==PID== Profiling result:' section")
    rest = text[m.end():]
    parts = re.split(r"==\d+== API calls:", rest, maxsplit=1)
    prof = _nvprof_rows(parts[0])
    api = _nvprof_rows(parts[1]) if len(parts) > 1 else []
    # newer nvprof prints both tables under "Profiling result:" with an "API calls:" label
    if not api:
        gpu_part, sep, api_part = parts[0].partition("API calls:")
        if sep:
            prof, api = _nvprof_rows(gpu_part), _nvprof_rows(api_part)
    return prof, api


# ----------------------------------------------------------------------------- rocprofv3
def parse_rocprof_stats_csv(path: str) -> List[dict]:
    """Rows of a rocprofv3 ``*_stats.csv`` in the reference schema (seconds)."""
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            try:
                rows.append({
                    "TimePerc": float(r["Percentage"]),
                    "Time": float(r["TotalDurationNs"]) * 1e-9,
                    "NumCalls": int(r["Calls"]),
                    "AvgCallTime": float(r["AverageNs"]) * 1e-9,
                    "MinCallTime": float(r["MinNs"]) * 1e-9,
                    "MaxCallTime": float(r["MaxNs"]) * 1e-9,
                    "CallName": r["Name"],
                })
            except (KeyError, ValueError):
                continue
    rows.sort(key=lambda r: -r["Time"])
    return rows


def parse_rocprof_dir(path: str) -> Tuple[List[dict], List[dict]]:
    """(kernel rows, API rows) from a rocprofv3 output directory (searched recursively)."""
    kern = sorted(glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True))
    if not kern:
        raise ValueError(f"no *kernel_stats.csv under {path}")
    prof = []
    for k in kern:
        prof += parse_rocprof_stats_csv(k)
    api = []
    for a in sorted(glob.glob(os.path.join(path, "**", "*hip_api_stats.csv"), recursive=True)):
        api += parse_rocprof_stats_csv(a)
    return prof, api


def write_rows(path: str, rows: Iterable[dict]) -> None:
    """CSV with a leading unnamed index column, like ``DataFrame.to_csv`` in the reference."""
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow([""] + COLUMNS)
        for i, r in enumerate(rows):
            w.writerow([i] + [r[c] for c in COLUMNS])


def compile_entry(entry: str, output_dir: str) -> int:
    """Process one log file / rocprof dir.  Returns 1 ok, -1 skipped, -2 unparsable
    (the reference's return codes, `scripts/compileResults.py:45-46,66-67`)."""
    name = os.path.basename(entry.rstrip("/"))
    if os.path.isdir(entry):
        stem = name
        try:
            prof, api = parse_rocprof_dir(entry)
        except ValueError:
            return -2
    elif name.endswith(".log"):
        stem = name[:-4]
        with open(entry, errors="replace") as f:
            text = f.read()
        try:
            prof, api = parse_nvprof_text(text)
        except ValueError:
            return -2
    else:
        return -1
    if parse_config_name(stem) is None:
        return -1
    os.makedirs(output_dir, exist_ok=True)
    write_rows(os.path.join(output_dir, f"profling_result_{stem}.csv"), prof)
    write_rows(os.path.join(output_dir, f"API_calls_{stem}.csv"), api)
    return 1


def summarize(input_dir: str) -> List[dict]:
    """One row per configuration: config columns + total GPU kernel time + top kernel."""
    out = []
    for entry in sorted(os.listdir(input_dir)):
        cfg = parse_config_name(entry)
        if cfg is None:
            continue
        p = os.path.join(input_dir, entry)
        try:
            prof, _ = parse_rocprof_dir(p) if os.path.isdir(p) else parse_nvprof_text(open(p).read())
        except (ValueError, OSError):
            continue
        tot = sum(r["Time"] for r in prof)
        top = max(prof, key=lambda r: r["Time"]) if prof else None
        out.append(dict(cfg, kernel_time_s=tot, n_kernels=sum(r["NumCalls"] for r in prof),
                        top_kernel=top["CallName"] if top else "",
                        top_kernel_time_s=top["Time"] if top else 0.0))
    return out
