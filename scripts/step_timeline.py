#!/usr/bin/env python3
"""Kernel timeline of the last steps of a traced run (rocprofv3 --kernel-trace CSV): every
dispatch with its start (from the step's first kernel), duration and the idle gap before it,
split into steps at each dispatch whose name matches <step regex> (the assign kernel).

    python3 scripts/step_timeline.py <rocprofv3 -d dir> <step regex> [steps to show]"""
import csv
import glob
import re
import sys


def main(root, pat, nshow=3):
    f = glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(f)))
    rx = re.compile(pat)
    starts = [i for i, r in enumerate(rows) if rx.search(r[2])]
    for si in range(max(0, len(starts) - nshow - 1), len(starts) - 1):
        a, b = starts[si], starts[si + 1]
        t0 = rows[a][0]
        busy = sum(rows[i][1] - rows[i][0] for i in range(a, b))
        print(f"-- step {si}: {(rows[b][0] - t0) / 1e3:.1f} us start to start, kernels {busy / 1e3:.1f} us")
        prev_end = None
        for i in range(a, b):
            s, e, n = rows[i]
            gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
            nm = re.sub(r"\(.*", "", n).replace("void ", "")[:70]
            print(f"   +{(s - t0) / 1e3:8.1f} us  {(e - s) / 1e3:8.1f} us  gap {gap:6.1f}  {nm}")
            prev_end = e


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 3)
