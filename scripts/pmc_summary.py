#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs: per kernel name, mean of each counter over dispatches."""
import collections
import csv
import glob
import re
import sys


def short(name):
    m = re.search(r"(tdc::(?:\w+::)*\w+(<[^>]*>)?|\w+_kernel\w*)", name)
    return (m.group(1) if m else name)[:70]


def main(root):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        disp = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Kernel_Name"])
            disp[key][r["Counter_Name"]] = disp[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for (d, k), cs in disp.items():
            for c, v in cs.items():
                per[short(k)][c].append(v)
    for k, cs in sorted(per.items()):
        print(k)
        for c, vs in sorted(cs.items()):
            print(f"    {c:38s} {sum(vs)/len(vs):14.4g}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
