#!/usr/bin/env python3
"""Summaries of tools/evidence.sh output (gpurun_out/TAG/), the numbers profiles/ cites.

  summarize.py stats   DIR            per-kernel calls / average / total from stats_*/run_kernel_stats.csv
  summarize.py traffic DIR WORKLOAD [launches_per_step]
        HBM bytes per launch of every kernel from fetch_W/ and write_W/ (rocprofv3 --pmc, kernel
        trace): FETCH_SIZE x 2 + WRITE_SIZE (the gfx950 correction of MI355X_MICROARCH.md's HBM
        section: FETCH_SIZE counts half the bytes of 128-byte streaming reads), KB x 1024.  With
        launches_per_step, also the bytes one bench step moves (all kernels of the step).
  summarize.py sq      DIR WORKLOAD   SQ counters per kernel (sq_W/, sq2_W/): averages per launch and
        the ratios DESIGN.md quotes (VALU / MFMA busy per wave cycle, LDS bank-conflict share).
Output is JSON on stdout."""
import collections
import csv
import glob
import json
import os
import sys


def short(name):
    base = name.replace("(anonymous namespace)::", "").split("(")[0]
    return base.replace("void ", "").replace("jw::", "")[:110]


def in_step(kernel):  # the bench's input generation (setup, untimed) is not part of a step
    return "synth_uniform" not in kernel


def counters(path):
    """{kernel: {counter: [values per dispatch]}} of one --pmc pass directory."""
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            out[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def stats(d):
    res = {}
    for f in sorted(glob.glob(os.path.join(d, "stats_*", "**", "*kernel_stats.csv"), recursive=True)):
        key = os.path.relpath(f, d).split(os.sep)[0]
        rows = []
        for r in csv.DictReader(open(f)):
            rows.append({"kernel": short(r["Name"]), "calls": int(r["Calls"]),
                         "avg_us": round(float(r["AverageNs"]) / 1e3, 2),
                         "total_ms": round(float(r["TotalDurationNs"]) / 1e6, 3),
                         "pct": round(float(r["Percentage"]), 2)})
        res[key] = rows
    return res


def traffic(d, w, per_step=None):
    fe, wr = counters(os.path.join(d, f"fetch_{w}")), counters(os.path.join(d, f"write_{w}"))
    res, step = {}, 0.0
    for k in fe:
        f = fe[k].get("FETCH_SIZE", [])
        s = wr.get(k, {}).get("WRITE_SIZE", [])
        if not f or not s:
            continue
        fb = sum(f) / len(f) * 1024 * 2
        wb = sum(s) / len(s) * 1024
        res[k] = {"launches": len(f), "fetch_x2_bytes": fb, "write_bytes": wb, "bytes": fb + wb}
        if in_step(k):
            step += (sum(f) * 2 + sum(s)) * 1024
    out = {"per_launch": res}
    if per_step:
        # all dispatches of the run = (warmup + steps) bench steps; report one step's worth
        out["bytes_per_step"] = step / float(per_step)
    return out


def sq(d, w):
    res = {}
    for sub in (f"sq_{w}", f"sq2_{w}"):
        for k, cs in counters(os.path.join(d, sub)).items():
            e = res.setdefault(k, {})
            for c, v in cs.items():
                e[c] = sum(v) / len(v)
    for k, e in res.items():
        wc = e.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_ACTIVE_INST_VALU", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAIT_INST_ANY",
                      "SQ_ACTIVE_INST_ANY"):
                if c in e:
                    e[c + "/WAVE_CYCLES"] = round(e[c] / wc, 4)
        if e.get("SQ_LDS_IDX_ACTIVE"):
            e["LDS_BANK_CONFLICT_share"] = round(e.get("SQ_LDS_BANK_CONFLICT", 0) / e["SQ_LDS_IDX_ACTIVE"], 4)
    return res


if __name__ == "__main__":
    mode, d = sys.argv[1], sys.argv[2]
    if mode == "stats":
        out = stats(d)
    elif mode == "traffic":
        out = traffic(d, sys.argv[3], int(sys.argv[4]) if len(sys.argv) > 4 else None)
    else:
        out = sq(d, sys.argv[3])
    json.dump(out, sys.stdout, indent=1)
    print()
