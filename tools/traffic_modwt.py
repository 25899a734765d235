#!/usr/bin/env python3
"""HBM traffic per launch of the MODWT kernels from tools/pmc.sh passes (p1 = FETCH_SIZE,
p2 = WRITE_SIZE, separate runs of bench.py): FETCH_SIZE x 2 (gfx950 correction,
MI355X_MICROARCH.md HBM section) + WRITE_SIZE, KB units x 1024, averaged over launches.
Usage: tools/traffic_modwt.py KEY gpurun_out/pmc_TAG [profiles/modwt_pmc_traffic.json]
merges {KEY: {kernel: bytes}} into the traffic file (KEY = wavelet/J/N/B/arith, as bench.py)."""
import collections
import csv
import json
import os
import sys

key, d = sys.argv[1], sys.argv[2]
path = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                          "modwt_pmc_traffic.json")
per = {}
for sub, c, mul in (("p1", "FETCH_SIZE", 2.0), ("p2", "WRITE_SIZE", 1.0)):
    disp = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f"{d}/{sub}/run_counter_collection.csv")):
        if r["Counter_Name"] != c or "modwt_" not in r["Kernel_Name"]:
            continue
        disp[r["Dispatch_Id"]] += float(r["Counter_Value"]) * 1024.0 * mul
        names[r["Dispatch_Id"]] = r["Kernel_Name"].split("<")[0].split("(")[0].split("::")[-1]
    acc = collections.defaultdict(list)
    for i, v in disp.items():
        acc[names[i]].append(v)
    for n, vs in acc.items():
        per.setdefault(n, 0.0)
        per[n] += sum(vs) / len(vs)
tr = json.load(open(path)) if os.path.exists(path) else {}
tr[key] = {n: int(round(v)) for n, v in per.items()}
tr.setdefault("_source_r03", f"{d} (tools/pmc.sh passes 1-2; tools/traffic_modwt.py)")
json.dump(tr, open(path, "w"), indent=1)
print(key, tr[key])
