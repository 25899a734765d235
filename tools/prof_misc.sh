#!/bin/bash
# Kernel stats (rocprofv3 --kernel-trace --stats) of the FWT-2D bench in both contracts and of
# JWave's default MODWT path (AUTO, STRICT) at cfg2 geometry x 16.  Usage: TAG
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/profmisc_$1"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/$name" -o run --output-format csv -- "$@" > "$O/$name.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -5 "$O/$name.log"; exit $rc; }
  python3 - "$O/$name/run_kernel_stats.csv" "$name" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "synth" in r["Name"] or float(r["Percentage"]) < 0.5:
        continue
    print(sys.argv[2], r["Name"][:90], r["Calls"], "avg_us %.1f" % (float(r["AverageNs"]) / 1e3))
PY
}
run fwt2d_fma python3 "$R/bench.py" --workload fwt2d --steps 3 --warmup 1 --no-cpu-baseline --no-check
run fwt2d_strict python3 "$R/bench.py" --workload fwt2d --steps 3 --warmup 1 --no-cpu-baseline --no-check --arith strict
run auto_strict python3 "$R/tools/modwt_time.py" --method auto --arith strict --reps 2
