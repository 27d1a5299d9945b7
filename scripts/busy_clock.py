#!/usr/bin/env python3
"""Per-dispatch MFMA busy fraction and shader clock from one rocprofv3 run that collected
GRBM_GUI_ACTIVE + SQ_VALU_MFMA_BUSY_CYCLES with --kernel-trace (scripts/pmc_mfma_busy.txt):

    busy  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
    clock = (GRBM_GUI_ACTIVE / 8) / dispatch duration

    python3 scripts/busy_clock.py <rocprofv3 -d dir> <kernel regex> [flop per dispatch]

Used for docs/PERF_NOTES.md (round 6, "MFMA busy against the clock"): under dense MFMA load
the chip lowers its clock as the busy fraction rises, so busy alone does not rank kernels."""
import collections
import csv
import glob
import re
import statistics
import sys


def main(root, pat, flop=0.0):
    rx = re.compile(pat)
    cnt = collections.defaultdict(dict)
    name = {}
    ts = {}
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if not rx.search(r["Kernel_Name"]):
                continue
            d = int(r["Dispatch_Id"])
            cnt[d][r["Counter_Name"]] = cnt[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            name[d] = r["Kernel_Name"]
            if "Start_Timestamp" in r and r["Start_Timestamp"]:
                ts[d] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            if d in cnt:
                ts[d] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    rows = []
    for d in sorted(cnt):
        c = cnt[d]
        if d not in ts or "GRBM_GUI_ACTIVE" not in c:
            continue
        ms = (ts[d][1] - ts[d][0]) / 1e6
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (cyc * 1024)
        ghz = cyc / (ms * 1e6)
        rows.append((d, ms, busy, ghz))
        pf = f"  {flop / ms / 1e12:6.3f} PF/s" if flop else ""
        print(f"dispatch {d:6d}  {ms:9.3f} ms  busy {busy:5.3f}  clock {ghz:5.3f} GHz  "
              f"busy x clock {busy * ghz:5.3f}{pf}")
    if rows:
        k = name[rows[0][0]]
        print(f"{k[:110]}\n  {len(rows)} dispatches; median {statistics.median(r[1] for r in rows):.3f} ms, "
              f"busy {statistics.median(r[2] for r in rows):.3f}, "
              f"clock {statistics.median(r[3] for r in rows):.3f} GHz, "
              f"busy x clock {statistics.median(r[2] * r[3] for r in rows):.3f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], float(sys.argv[3]) if len(sys.argv) > 3 else 0.0)
