#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs: per kernel, median over dispatches of each
counter (grouped by the ablation variant order in which kernels ran)."""
import csv
import glob
import statistics
import sys
from collections import defaultdict

root = sys.argv[1]
per = defaultdict(lambda: defaultdict(list))   # (kernel, dispatch) -> counter -> vals
for f in glob.glob(root + "/p*/pmc_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "qhuff" not in r["Kernel_Name"]:
            continue
        k = "enc" if "encode" in r["Kernel_Name"] else "dec"
        per[(f, k, int(r["Dispatch_Id"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
# order dispatches within each file; split into variants of 25 iterations
out = defaultdict(lambda: defaultdict(list))
for (f, k, d), cs in per.items():
    for c, v in cs.items():
        out[(f, k)][c].append((d, sum(v)))
res = defaultdict(dict)
for (f, k), cs in out.items():
    for c, lst in cs.items():
        lst.sort()
        vals = [v for _, v in lst]
        nvar = max(1, len(vals) // 25)
        for vi in range(nvar):
            chunk = vals[vi * 25 + 5:(vi + 1) * 25]
            res[(k, vi)][c] = statistics.median(chunk) if chunk else float("nan")
for key in sorted(res):
    print(key, {c: ("%.4g" % v) for c, v in sorted(res[key].items())})
