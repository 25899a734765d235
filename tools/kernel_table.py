#!/usr/bin/env python3
"""One table per evidence directory: every kernel's launches per repetition, average duration,
HBM bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE, tools/summarize.py traffic) and the rate those
bytes give.  Needs the stats_W and fetch_W / write_W passes of tools/evidence.sh in DIR.

  kernel_table.py DIR WORKLOAD REPS      (REPS: calls of the workload in the profiled run)

The FETCH_SIZE x 2 correction holds for 128-byte streaming reads; for 64-byte pieces it counts
double (MI355X_MICROARCH.md), so those kernels' rates read high."""
import csv
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def short(n):
    return n.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("jw::", "")[:110]


def main():
    d, w, reps = sys.argv[1], sys.argv[2], float(sys.argv[3])
    rows = list(csv.DictReader(open(os.path.join(d, f"stats_{w}", "run_kernel_stats.csv"))))
    t = json.loads(subprocess.check_output(
        [sys.executable, os.path.join(HERE, "summarize.py"), "traffic", d, w]))["per_launch"]
    tot = 0.0
    for r in rows:
        n = short(r["Name"])
        if any(k in n for k in ("synth", "distribution", "copyBuffer")):
            continue
        avg = float(r["AverageNs"]) / 1e3
        tr = t.get(n, {})
        b = tr.get("bytes", 0)
        tot += float(r["TotalDurationNs"]) / 1e6 / reps
        print(f"{n[:88]:90s} {int(r['Calls']) / reps:6.1f}/rep {avg:8.1f} us  "
              f"fetch {tr.get('fetch_x2_bytes', 0) / 1e6:8.1f} MB write {tr.get('write_bytes', 0) / 1e6:8.1f} MB  "
              f"{b / avg / 1e6 if avg else 0:5.2f} TB/s")
    print("total ms/rep", round(tot, 3))


if __name__ == "__main__":
    main()
