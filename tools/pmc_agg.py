"""Aggregate rocprofv3 counter_collection.csv files: per kernel name, the mean per dispatch of
every counter (summed over the dimension instances of a dispatch).  Usage:
    python tools/pmc_agg.py <dir-or-csv>... [--kernel REGEX]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def load(paths):
    per = defaultdict(lambda: defaultdict(float))   # (kernel, dispatch) -> counter -> value
    for p in paths:
        for row in csv.DictReader(open(p)):
            k = (row["Kernel_Name"], row.get("Dispatch_Id") or row.get("Correlation_Id"))
            per[k][row["Counter_Name"]] += float(row["Counter_Value"])
    agg = defaultdict(lambda: defaultdict(list))
    for (name, _), cs in per.items():
        for c, v in cs.items():
            agg[name][c].append(v)
    return agg


if __name__ == "__main__":
    argv = sys.argv[1:]
    rx = None
    if "--kernel" in argv:
        i = argv.index("--kernel")
        rx = re.compile(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    args = argv
    paths = []
    for a in args:
        paths += sorted(glob.glob(os.path.join(a, "*counter_collection.csv"))) if os.path.isdir(a) else [a]
    agg = load(paths)
    for name in sorted(agg):
        if rx and not rx.search(name):
            continue
        print(name)
        for c, v in sorted(agg[name].items()):
            print("   %-26s n=%4d mean=%.4g" % (c, len(v), sum(v) / len(v)))
