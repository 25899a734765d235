#!/usr/bin/env python3
"""Average each PMC counter per MODWT kernel over all dispatches of a tools/pmc.sh run."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
res = collections.defaultdict(dict)
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "modwt" not in k and "fwt" not in k and "cwt" not in k and "inv_nomem" not in k:
            continue
        k = k.split("(")[0].replace("void ", "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        for c, x in v.items():
            res[k][c] = sum(x) / len(x)
for k in res:
    print(k)
    for c, v in sorted(res[k].items()):
        print(f"   {c:40s} {v:.4g}")
