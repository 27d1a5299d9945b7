#!/usr/bin/env python3
"""Row-by-row comparison of MI355X sweep logs with the reference's executions_log.csv.

    python scripts/compare_with_reference.py \
        --ours fp64=results/like_for_like_r03/executions_log_mi355x_fp64.csv \
        --ours fp32=results/like_for_like_r03/executions_log_mi355x_fp32.csv \
        --reference /root/reference/scripts/executions_log.csv > COMPARISON.md

Both logs have the reference's 10-column schema (`scripts/distribuitedClustering.py:33-35`).
points assigned/s = n_obs * n_iter / computation_time (BASELINE.md's derivation).  Every
MI355X row is set against the reference row of the SAME (method, K, n_obs, GPU count) --
the like-for-like cell of `scripts/executions_log.csv` -- and against the reference's best
GPU count for that (method, K, n_obs).  Reference cells that failed (InternalError: the
[N/G, K, D] fp64 distance tiles out of memory) are shown with their line numbers.
A bare ``--ours path`` is labelled by its file name.
"""
import argparse
import csv
import os
from collections import defaultdict


def rows(path):
    with open(path, newline="") as f:
        for i, r in enumerate(csv.DictReader(f), start=2):
            r["_line"] = i
            yield r


def num(v):
    try:
        return float(v)
    except (TypeError, ValueError):
        return None


def pps(r):
    ct = num(r["computation_time"])
    it = int(r["n_iter"]) if str(r["n_iter"]).isdigit() else 0
    return int(r["n_obs"]) * it / ct if ct else None


def ref_cell(cands):
    """(text, points/s or None) of the fastest successful reference row among cands."""
    ok = [x for x in cands if num(x["computation_time"])]
    if ok:
        b = min(ok, key=lambda x: num(x["computation_time"]))
        return (f"{b['num_GPUs']} GPUs, line {b['_line']}: {num(b['computation_time']):.3f} s, "
                f"{pps(b) / 1e6:.1f} M/s", pps(b))
    if not cands:
        return "no row", None
    fails = sorted({x["setup_time"] for x in cands})
    lines = sorted(x["_line"] for x in cands)
    span = f"line {lines[0]}" if len(lines) == 1 else f"lines {lines[0]}-{lines[-1]}"
    return f"failed ({', '.join(fails)}; {span})", None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ours", required=True, action="append",
                    help="LABEL=path (repeatable; e.g. fp64=..., fp32=...)")
    ap.add_argument("--reference", required=True)
    a = ap.parse_args()
    ref = defaultdict(list)
    for r in rows(a.reference):
        key = (r["method_name"].replace("distribuited", "distributed"), int(r["K"]), int(r["n_obs"]))
        ref[key].append(r)
    print("| method | K | n_obs | GPUs | dtype | MI355X computation_time s | MI355X points/s | "
          "reference, same GPU count | speed-up (same GPUs) | reference, best GPU count | "
          "speed-up (best) |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    summary = defaultdict(list)
    for spec in a.ours:
        label, path = spec.split("=", 1) if "=" in spec else (os.path.basename(spec), spec)
        for r in rows(path):
            m, k, n, g = r["method_name"], int(r["K"]), int(r["n_obs"]), int(r["num_GPUs"])
            ours = pps(r)
            cands = ref.get((m, k, n), [])
            same_txt, same_p = ref_cell([x for x in cands if int(x["num_GPUs"]) == g])
            best_txt, best_p = ref_cell(cands)
            sp_same = f"{ours / same_p:.0f}x" if ours and same_p else ("ref failed" if ours else "-")
            sp_best = f"{ours / best_p:.0f}x" if ours and best_p else ("ref failed" if ours else "-")
            if ours and best_p:
                summary[(label, m)].append(ours / best_p)
            ot = (f"{num(r['computation_time']):.4f} | {ours / 1e9:.2f} G" if ours
                  else f"{r['computation_time']} | -")
            print(f"| {m} | {k} | {n:,} | {g} | {label} | {ot} | {same_txt} | {sp_same} | "
                  f"{best_txt} | {sp_best} |")
    if summary:
        print()
        print("| dtype | method | rows with a reference number | speed-up over the reference's best "
              "GPU count: min / max |")
        print("|---|---|---|---|")
        for (label, m), v in sorted(summary.items()):
            print(f"| {label} | {m} | {len(v)} | {min(v):.0f}x / {max(v):.0f}x |")


if __name__ == "__main__":
    main()
