#!/usr/bin/env python3
"""HBM traffic per bench step from tools/pmc_traffic.sh output: every kernel launched by one
step (the warmup and the timed step are the same work, so half of all launches of the step's
kernels), FETCH_SIZE x 2 (gfx950 correction, MI355X_MICROARCH.md HBM section) + WRITE_SIZE,
in bytes.  Usage: tools/traffic_summary.py gpurun_out/pmctraffic_TAG > profiles/...json"""
import collections
import csv
import json
import sys

d = sys.argv[1]
out = {}
STEP_KERNELS = {"cwt": ("pass512", "cwt_band"), "fwt2d": ("fwt_",)}
for w, keys in STEP_KERNELS.items():
    tot = {}
    per_kernel = collections.defaultdict(float)
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        s = 0.0
        for r in csv.DictReader(open(f"{d}/{w}_{c}/run_counter_collection.csv")):
            if any(k in r["Kernel_Name"] for k in keys):
                v = float(r["Counter_Value"]) * 1024.0 * (2.0 if c == "FETCH_SIZE" else 1.0)
                s += v
                name = r["Kernel_Name"].split("(")[0][-60:]
                per_kernel[name] += v / 2
        tot[c] = s / 2  # warmup step + timed step
    out[w] = {"bytes_per_step": tot["FETCH_SIZE"] + tot["WRITE_SIZE"],
              "fetch_bytes_x2": tot["FETCH_SIZE"], "write_bytes": tot["WRITE_SIZE"],
              "per_kernel_bytes": dict(per_kernel)}
out["_source"] = (f"{d}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate runs of bench.py "
                  "--steps 1 --warmup 1 (KB units); FETCH_SIZE x2 per the gfx950 correction")
print(json.dumps(out, indent=1))
