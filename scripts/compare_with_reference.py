#!/usr/bin/env python3
"""Row-by-row comparison of an MI355X sweep log with the reference's executions_log.csv.

    python scripts/compare_with_reference.py --ours results/like_for_like_r02/executions_log_mi355x.csv \
        --reference /root/reference/scripts/executions_log.csv > results/like_for_like_r02/COMPARISON.md

Both logs have the reference's 10-column schema (`scripts/distribuitedClustering.py:33-35`).
points assigned/s = n_obs * n_iter / computation_time (BASELINE.md's derivation).  For every
(method, K, n_obs) the reference's best GPU count is shown next to ours; configurations
whose reference rows all failed (InternalError, the [N/G, K, D] fp64 tiles out of memory)
are listed with the failure.
"""
import argparse
import csv
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ours", required=True)
    ap.add_argument("--reference", required=True)
    a = ap.parse_args()
    ref = defaultdict(list)
    for r in rows(a.reference):
        key = (r["method_name"].replace("distribuited", "distributed"), int(r["K"]), int(r["n_obs"]))
        ref[key].append(r)
    print("| method | K | n_obs | MI355X GPUs | MI355X computation_time s | MI355X points/s | "
          "reference best (GPUs, CSV line) | reference computation_time s | reference points/s | speed-up |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for r in rows(a.ours):
        m, k, n = r["method_name"], int(r["K"]), int(r["n_obs"])
        ct = num(r["computation_time"])
        it = int(r["n_iter"]) if r["n_iter"].isdigit() else 0
        pps = n * it / ct if ct else None
        ok = [x for x in ref.get((m, k, n), []) if num(x["computation_time"])]
        if ok:
            b = min(ok, key=lambda x: num(x["computation_time"]))
            rct = num(b["computation_time"])
            rpps = n * int(b["n_iter"]) / rct
            refcol = f"{b['num_GPUs']} GPUs (line {b['_line']}) | {rct:.3f} | {rpps / 1e6:.1f} M"
            sp = f"{pps / rpps:.0f}x" if pps else "-"
        else:
            fails = sorted({x["setup_time"] for x in ref.get((m, k, n), [])})
            lines = [x["_line"] for x in ref.get((m, k, n), [])]
            span = f"lines {min(lines)}-{max(lines)}" if lines else "no rows"
            refcol = f"all {len(lines)} runs failed ({', '.join(fails)}; {span}) | - | -"
            sp = "ref failed"
        ours = f"{ct:.4f} | {pps / 1e9:.2f} G" if pps else f"{r['computation_time']} | -"
        print(f"| {m} | {k} | {n:,} | {r['num_GPUs']} | {ours} | {refcol} | {sp} |")


if __name__ == "__main__":
    main()
