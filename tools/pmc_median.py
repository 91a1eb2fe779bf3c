#!/usr/bin/env python3
"""Median per dispatch of each PMC counter, per qhuff kernel, over the CSVs
under a tools/pmc_pass.sh output directory; plus derived ratios."""
import csv
import glob
import statistics
import sys
from collections import defaultdict

root = sys.argv[1]
per = defaultdict(lambda: defaultdict(float))   # (kernel, file, dispatch) -> counter -> sum
for f in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "qhuff" not in r["Kernel_Name"]:
            continue
        k = "enc" if "encode" in r["Kernel_Name"] else "dec"
        per[(k, f, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
res = defaultdict(lambda: defaultdict(list))
for (k, f, d), cs in per.items():
    for c, v in cs.items():
        res[k][c].append(v)
for k in sorted(res):
    m = {c: statistics.median(v) for c, v in res[k].items()}
    print(k, " ".join("%s=%.4g" % (c, v) for c, v in sorted(m.items())))
    w = m.get("SQ_WAVES", 0)
    if w:
        print("   per wave: VALU %.0f SALU %.0f LDS %.0f BRANCH %.0f  wave-cycles %.0f"
              % (m.get("SQ_INSTS_VALU", 0) / w, m.get("SQ_INSTS_SALU", 0) / w,
                 m.get("SQ_INSTS_LDS", 0) / w, m.get("SQ_INSTS_BRANCH", 0) / w,
                 m.get("SQ_WAVE_CYCLES", 0) / w))
    if m.get("SQ_WAVE_CYCLES"):
        wc = m["SQ_WAVE_CYCLES"]
        print("   of wave-cycles: WAIT_ANY %.2f WAIT_INST_ANY %.2f ACTIVE_ANY %.2f "
              "(VALU %.2f LDS %.2f SCA %.2f) WAIT_INST_LDS %.2f"
              % tuple(m.get(c, 0) / wc for c in (
                  "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                  "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_LDS")))
