#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs into per-kernel totals (small JSON for profiles/)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def summarise(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    agg = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r.get("Kernel_Name", "?")[:90]
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r.get("Dispatch_Id"))
    out = {k: dict(v, dispatches=len(disp[k])) for k, v in agg.items()}
    tot = defaultdict(float)
    for v in out.values():
        for c, x in v.items():
            tot[c] += x
    return {"per_kernel": out, "total": dict(tot)}


if __name__ == "__main__":
    res = {os.path.basename(d.rstrip("/")): summarise(d) for d in sys.argv[1:-1]}
    with open(sys.argv[-1], "w") as f:
        json.dump(res, f, indent=1)
    for name, r in res.items():
        print(name, json.dumps({k: round(v) for k, v in r["total"].items()}))
