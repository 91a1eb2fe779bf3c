#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py into
profiles/pmc_<tag>.json: HBM bytes per launch for each qhuff kernel.

Correction (MI355X_MICROARCH.md, section HBM): on gfx950 FETCH_SIZE reports
half the bytes of a wide (16 B/lane) coalesced streaming read, so the read
side is doubled; WRITE_SIZE reads exact for 16-B streaming stores.  Both
counters are in KiB.  Usage: pmc_summary.py FETCH_DIR WRITE_DIR N OUT.json
"""
import csv
import glob
import json
import statistics
import sys


def per_kernel(d, counter):
    vals = {}
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter or "qhuff" not in r["Kernel_Name"]:
                continue
            name = r["Kernel_Name"]
            k = next((x for x in ("qhuff_encode_kernel", "qhuff_decode_kernel",
                                  "qhuff_hash_kernel") if x in name), None)
            if k is None:
                continue
            key = (k, r["Dispatch_Id"])
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    out = {}
    for (k, _), v in vals.items():
        out.setdefault(k, []).append(v)
    return {k: statistics.median(v) for k, v in out.items()}


def main():
    fdir, wdir, n, outp = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    fetch = per_kernel(fdir, "FETCH_SIZE")
    write = per_kernel(wdir, "WRITE_SIZE")
    res = {"note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KiB->B",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        fb = fetch.get(k, 0.0) * 1024 * 2
        wb = write.get(k, 0.0) * 1024
        res["kernels"][k] = {"n": n // 2 if "hash" in k else n, "fetch_bytes_raw": fetch.get(k, 0.0) * 1024,
                             "fetch_bytes": fb, "write_bytes": wb,
                             "hbm_bytes_per_launch": int(fb + wb)}
    json.dump(res, open(outp, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
