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
        if not any(s in k for s in ("modwt", "fwt", "cwt", "inv_nomem", "pass512", "pass_generic", "psi_table", "jf::kp")):
            continue
        k = k.replace("(anonymous namespace)", "anon").split("(")[0].replace("void ", "")[:90]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        for c, x in v.items():
            res[k][c] = sum(x) / len(x)
for k in res:
    print(k)
    for c, v in sorted(res[k].items()):
        print(f"   {c:40s} {v:.4g}")
